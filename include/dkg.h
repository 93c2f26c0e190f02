/*
 * dkg.h — C ABI of the MI355X-native Discrete Knowledge Gradient hot path.
 *
 * The reference (quasirandom/decoupled-kg, pure Python) computes the discrete
 * multi-objective KG in
 *   src/decoupledbo/modules/acquisition/discretekg.py
 *     DiscreteKnowledgeGradient.forward                       :131-159
 *     calculate_discrete_kg                                    :162-235
 *     calculate_discrete_kg_conditioning_on_single_output      :238-338
 *     calculate_epigraph_indices                               :341-412
 *     calculate_expected_value_of_piecewise_linear_function    :415-452
 * on top of BoTorch/GPyTorch exact GP posteriors (model.posterior at
 * :182-185 and :275-284; model family src/decoupledbo/modules/model/factory.py).
 *
 * This library replaces that arithmetic with hand-written HIP kernels for
 * gfx950.  Plain pointers and sizes only; every pointer marked "device" is a
 * device allocation owned by the caller; every entry point is stream ordered
 * on `stream` (a hipStream_t, NULL = legacy default stream) and never
 * synchronises unless its name says "timed".  Status codes instead of
 * exceptions; dkg_last_error() returns a thread-local message.
 *
 * Data layout in HBM (see DESIGN.md "Data layout"):
 *   n_pad(n) = n rounded up to a multiple of 16.
 *   A "fragment-packed" matrix P (rows x n, rows padded to 16, KB = n_pad/4
 *   k-blocks) is stored pair-packed:
 *     F[t][j][l][h] = P[16 t + (l & 15)][4 (2 j + h) + (l >> 4)],
 *   t < rows_pad/16, j < KB/2, l < 64, h < 2 — the per-lane operand order of
 *   v_mfma_f64_16x16x4_f64 for k-blocks 2j and 2j+1 side by side, so one
 *   coalesced 16-byte-per-lane (1 KiB) load feeds two MFMAs.  Padding entries
 *   are zero.
 */
#ifndef DKG_AMD_DKG_H
#define DKG_AMD_DKG_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DKG_ABI_VERSION 8  /* 8: dkg_plan_forward_batches, dkg_plan_time_stage_batches; 7: DKG_PLAN_NO_CHAIN */
#define DKG_MAX_OUTPUTS 8   /* outputs (objectives) per model list */
#define DKG_MAX_DIM 16      /* input dimension d */

enum dkg_status {
  DKG_OK = 0,
  DKG_ERR_ARG = 1,          /* bad argument / shape (reference raises BotorchTensorDimensionError) */
  DKG_ERR_UNSUPPORTED = 2,  /* outside supported sizes (reference: UnsupportedError) */
  DKG_ERR_WORKSPACE = 3,    /* workspace too small */
  DKG_ERR_HIP = 4,          /* HIP runtime error */
  DKG_ERR_NO_LINES = 5,     /* no lines (reference: ValueError, discretekg.py:466-470) */
  DKG_ERR_NOT_PD = 6        /* covariance not positive definite after the jitter retries
                               (linear_operator psd_safe_cholesky raises NotPSDError) */
};

/* Covariance families of model/factory.py:116 (ScaleKernel(base)). */
enum dkg_kernel { DKG_MATERN12 = 0, DKG_MATERN32 = 1, DKG_MATERN52 = 2, DKG_RBF = 3 };

/* Fitted state of one output GP (one SingleTaskGP of the ModelListGP,
 * factory.py:63-88) plus its caches over the discretisation.  The caches are
 * the quantities GPyTorch keeps for exact prediction with fast_pred_var:
 * R = L^{-T} with L = chol(K_XX + noise I), alpha = (K_XX + noise I)^{-1}(y - c). */
typedef struct dkg_output {
  int32_t n;                 /* training points */
  int32_t kernel;            /* enum dkg_kernel */
  double outputscale;        /* ScaleKernel outputscale s */
  double noise;              /* likelihood noise variance (model space) */
  double mean_constant;      /* ConstantMean c */
  double y_mean, y_std;      /* Standardize(m=1) untransform (0, 1 if absent) */
  const double* inv_lengthscale; /* device [d]: 1 / ARD lengthscale */
  const double* train_x;     /* device [n x d] row-major (normalised inputs) */
  const double* alpha;       /* device [n_pad(n)], zero padded */
  const double* root_frag;   /* device, fragment-packed R^T (P[c][r] = R[r][c]), n_pad^2 */
  const double* disc_frag;   /* device, fragment-packed Q_D = K(D,X) R: N_pad x n_pad (nullable for dkg_cross_root) */
  const double* disc_mean;   /* device [N]: c + K(D,X) alpha, model space (nullable for dkg_cross_root) */
} dkg_output;

int dkg_abi_version(void);
const char* dkg_last_error(void);

/* Number of doubles of a fragment-packed (rows x n) matrix: n_pad(rows)*n_pad(n). */
size_t dkg_frag_elems(int rows, int n);

/* out[i*n2+j] = s*k(x1_i, x2_j) (+ diag_add on i==j when n1==n2).
 * Replaces the covariance evaluation of ScaleKernel(Matern|RBF) (factory.py:110-135,
 * GPyTorch Kernel.forward) used to build K_XX + noise I for the Cholesky. */
int dkg_kernel_matrix(const dkg_output* o, int d, const double* x1, int n1, const double* x2, int n2,
                      double diag_add, double* out, void* stream);

/* Bytes of device scratch dkg_prepare_output needs for n training points. */
size_t dkg_prepare_workspace(int n);

/* Fitted-state caches of one output computed on the device by the library's
 * own kernels (no rocSOLVER / rocBLAS): the quantities GPyTorch's exact
 * prediction caches behind model.posterior (discretekg.py:182-185, 275-284;
 * gpytorch DefaultPredictionStrategy, linear_operator psd_safe_cholesky):
 *   K = s k(X, X) + noise I (+ jitter I)
 *   L = chol(K): blocked right-looking Cholesky; when it fails, retried with
 *       absolute jitter 1e-8 * 10^i, i < max_tries (linear_operator's policy)
 *   R = L^{-T} (root_inv_decomposition), packed into root_frag
 *   alpha = K^{-1} (y - c)  (n_pad doubles, zero padded)
 * o: n, kernel, outputscale, noise, mean_constant, inv_lengthscale, train_x
 *    (alpha / root_frag / disc_* are ignored).  train_y: device [n] targets
 * (model space).  L: device [n x n], receives L (row-major, zero upper
 * triangle).  work: device scratch of dkg_prepare_workspace(n) bytes; on
 * return it starts with L^{-1} (row-major n x n).  jitter_used (host,
 * nullable): the absolute jitter that made K positive definite (0 if none).
 * Synchronises `stream` once per Cholesky attempt (the retry policy reads the
 * factorisation status).  DKG_ERR_NOT_PD if every attempt failed. */
int dkg_prepare_output(const dkg_output* o, int d, const double* train_y, int max_tries, double* L, void* work,
                       size_t work_bytes, double* alpha, double* root_frag, double* jitter_used, void* stream);

/* dkg_prepare_output for m outputs at once (host arrays of m per-output pointers): every launch of
 * the first Cholesky attempt and of the inverse carries all outputs (one workgroup column per output),
 * one synchronisation checks all the factorisations, and only outputs that failed are retried with
 * jitter, one by one.  Same results as m calls of dkg_prepare_output.  jitter_used: host [m]. */
int dkg_prepare_outputs(const dkg_output* outs, int m, int d, const double* const* train_y, int max_tries,
                        double* const* L, void* const* work, const size_t* work_bytes, double* const* alpha,
                        double* const* root_frag, double* jitter_used, void* stream);

/* Pack dense row-major R (n x n, device) into o->root_frag layout (device). */
int dkg_pack_root(const double* r, int n, double* root_frag, void* stream);

/* Q = K(x, X) R (fragment-packed, rows x n) and mean = c + K(x, X) alpha (model
 * space, nullable).  This is the test-train half of GPyTorch's exact
 * prediction (DefaultPredictionStrategy mean_cache / covar_cache products)
 * behind model.posterior (discretekg.py:182-185, :275-284).  With x = the
 * discretisation D it builds disc_frag / disc_mean. */
int dkg_cross_root(const dkg_output* o, int d, const double* x, int rows, double* q_frag,
                   double* mean, void* stream);

/* Bytes of scratch dkg_forward needs for (m outputs, N points, B candidates, S weights). */
size_t dkg_forward_workspace(const dkg_output* outs, int m, int N, int B, int S);

/* Discrete KG for B candidates: kg[b] = mean_j KG(xnew_b, w_j).
 * Replaces DiscreteKnowledgeGradient.forward (discretekg.py:131-159) with
 * target = -1 -> calculate_discrete_kg (:162-235, coupled evaluation),
 * target = t  -> calculate_discrete_kg_conditioning_on_single_output (:238-338).
 *   outs    : m output states (host array of structs holding device pointers)
 *   disc    : device [N x d] discretisation (x_discretisation)
 *   xnew    : device [B x d] candidates
 *   weights : device [S x m] linear scalarisation weights
 *   kg      : device [B] output
 *   kg_pairs: device [B x S] per-(candidate, scalarisation) KG, nullable
 *   workspace: device scratch of dkg_forward_workspace() bytes */
int dkg_forward(const dkg_output* outs, int m, int d, const double* disc, int N, const double* xnew,
                int B, const double* weights, int S, int target, double* kg, double* kg_pairs,
                void* workspace, size_t workspace_bytes, void* stream);

/* As dkg_forward, but records HIP events around each of the three kernels on
 * `stream`, synchronises, and returns their durations in ms:
 * stage_ms[0] = cross (K(x,X) R), [1] = posterior covariance GEMM, [2] = envelope + expectation. */
int dkg_forward_timed(const dkg_output* outs, int m, int d, const double* disc, int N, const double* xnew,
                      int B, const double* weights, int S, int target, double* kg, double* kg_pairs,
                      void* workspace, size_t workspace_bytes, void* stream, float* stage_ms);

/* ---- Plan API (the fast path) -------------------------------------------
 * A plan is everything a forward needs besides the candidates: the m output
 * states, the discretisation, the weights, the target and the workspace carve
 * for up to max_B candidates.  dkg_plan_init validates it, writes it to
 * `host_plan` (caller memory of dkg_plan_bytes() bytes, kept unchanged while
 * the plan is in use) and copies it to `dev_plan` (device memory of the same
 * size) on `stream`.  dkg_plan_forward then launches the three kernels with a
 * pointer to the device copy (no per-call host-to-device traffic).  The
 * disc/weights/workspace buffers must outlive the plan.  The weights are
 * frozen at dkg_plan_init: the staged envelope's intercept cache and each
 * scalarisation's top intercept (Plan::icpt / itop) are derived from them
 * there, so a caller that changes its weights builds a new plan (the Python
 * host passes the plan a copy of its weights and rebuilds on a change). */
/* Plan flags: DKG_PLAN_GRAD adds the gradient buffers (dkg_plan_forward_grad). */
#define DKG_PLAN_GRAD 1
/* DKG_PLAN_FORCE_WALK (test hook): the envelope stage takes its list-overflow
 * path (gift wrap over all lines) for every pair; same results, slower. */
#define DKG_PLAN_FORCE_WALK 2
/* DKG_PLAN_F32: the two contractions of the forward (Q_X = K(x,X) R and
 * Q_X . Q_D, BASELINE configs[4]'s "fp32 MFMA-bound stress") run in fp32 on
 * v_mfma_f32_16x16x4_f32 over fp32 copies of R and Q_D made at plan init; the
 * kernel evaluations, means, variances (fp64 sums of the fp32 Q_X squares),
 * the line build, envelope and expectation stay fp64.  Not a reference mode
 * (the reference is fp64 throughout, constants.py:8): results agree with the
 * fp64 plan to ~1e-3 relative when the noise is >= 1e-3 of the outputscale.
 * Forward only (not combinable with DKG_PLAN_GRAD). */
#define DKG_PLAN_F32 4
/* DKG_PLAN_FUSED: dkg_plan_forward launches the forward as ONE kernel whose cross,
 * covariance and envelope workgroups hand the stages on through arrival counters
 * (dkg_fused.h), instead of the three stage kernels; fp64 plans whose lines fit the
 * staged envelope (N + 1 <= 1088).  Same bits either way.  Not the default: on
 * MI355X an in-launch hand-off costs about what the kernel boundary it replaces
 * does, and the early-dispatched consumers slow the producers. */
#define DKG_PLAN_FUSED 8
/* DKG_PLAN_NO_CHAIN (test hook): the streaming envelope (N + 1 > 2112 lines, or line data beyond LDS)
 * filters without its sample chain: the extremes from the streamed lines, the quickhull refinement and
 * the walks of the list-overflow path for every pair; same results, slower. */
#define DKG_PLAN_NO_CHAIN 16
size_t dkg_plan_bytes(void);
size_t dkg_plan_workspace(const dkg_output* outs, int m, int d, int N, int max_B, int S, int flags);
int dkg_plan_init(const dkg_output* outs, int m, int d, const double* disc, int N, const double* weights, int S,
                  int target, int max_B, int flags, void* workspace, size_t workspace_bytes, void* host_plan,
                  void* dev_plan, void* stream);
/* kg[b] (and kg_pairs[b x S], nullable) for B <= max_B candidates xnew (device, B x d);
 * same result as dkg_forward with the plan's arguments.  One fused launch for a plan built
 * with DKG_PLAN_FUSED (a call given kg_pairs runs the three stages). */
int dkg_plan_forward(const void* host_plan, const void* dev_plan, const double* xnew, int B, double* kg,
                     double* kg_pairs, void* stream);
/* nbatch forward batches of B candidates in one launch per stage: xnew is device [nbatch][B][d], kg
 * device [nbatch][B], nbatch * B <= max_B.  kg[k][b] is bit-for-bit what dkg_plan_forward of batch k
 * alone writes (every candidate's result depends on its own x only, and the covariance blocks are the
 * ones a B-candidate forward takes), so this is nbatch dkg_plan_forward calls with 3 launches instead
 * of 3 * nbatch: the throughput form of the reference's per-batch forward (discretekg.py:131-159) when
 * a caller has several batches ready (bench.py's steps).  Always the three stage kernels (a fused plan
 * included). */
int dkg_plan_forward_batches(const void* host_plan, const void* dev_plan, const double* xnew, int B, int nbatch,
                             double* kg, void* stream);
/* As dkg_plan_forward with per-kernel HIP-event timings (synchronises): stage_ms[3]. */
int dkg_plan_forward_timed(const void* host_plan, const void* dev_plan, const double* xnew, int B, double* kg,
                           double* kg_pairs, void* stream, float* stage_ms);
/* Value and gradient (plan built with DKG_PLAN_GRAD): kg[b] as dkg_plan_forward
 * and dkg_dx[b*d + j] = d kg[b] / d xnew[b*d + j] (device, B x d).  Replaces
 * the autograd backward of DiscreteKnowledgeGradient.forward (discretekg.py:
 * 131-159; exercised by test_discretekg.py:110-135 and by optimize_acqf,
 * acquisition_optimisation_strategy.py:217-224, 259-266).  With the upper
 * envelope fixed (envelope theorem), per scalarisation
 *   dKG/dx = sum_{envelope lines e} [ (phi(c_L) - phi(c_R)) db_e/dx
 *                                      + (Phi(c_R) - Phi(c_L)) [e = 0] da_0/dx ]
 *            - [line 0 attains max a] da_0/dx,
 * where only the candidate's own line 0 intercept and the slopes depend on x. */
int dkg_plan_forward_grad(const void* host_plan, const void* dev_plan, const double* xnew, int B, double* kg,
                          double* dkg_dx, void* stream);
/* Largest B * d of dkg_plan_forward_grad_hostx. */
#define DKG_XARG_MAX 64
/* dkg_plan_forward_grad for candidates given in HOST memory (x_host[b*d + j], B * d <= DKG_XARG_MAX):
 * the candidates travel inside the first kernel's arguments instead of a host-to-device copy
 * (one copy fewer on the optimize_acqf L-BFGS-B path, batch_limit = 1: bo_loop.py:127-129), and
 * that kernel leaves them in x_dev (device, B x d) for the later kernels.  x_host may be reused as
 * soon as this returns.  out_host (nullable): pinned host memory of B * (d + 1) doubles that
 * receives [kg | dkg_dx], written by the envelope kernel itself (no copy after it); with out_host the
 * call synchronises the stream and returns with the results in place (one host call per L-BFGS-B
 * evaluation).  Same results, bit for bit, as dkg_plan_forward_grad on x_dev. */
int dkg_plan_forward_grad_hostx(const void* host_plan, const void* dev_plan, const double* x_host, double* x_dev,
                                int B, double* kg, double* dkg_dx, double* out_host, void* stream);
/* Envelope sizes of the plan's last forward that was given kg_pairs (same B):
 * out[b*S + j] = the number of upper-envelope lines of pair (b, j), i.e. the
 * len(indices) of calculate_epigraph_indices (discretekg.py:341-412); 1 when the
 * pair short-circuits (all |b| < 1e-9, :363-367).  Device int[B x S]; stream
 * ordered.  Diagnostics (log the envelope-size histogram). */
int dkg_plan_hull_sizes(const void* host_plan, int* out, int B, void* stream);
/* Hand-off status of the plan's fused launches (DKG_PLAN_FUSED) (stream ordered, synchronises):
 * *err = the OR of the bits of every in-launch wait that gave up since the last
 * reset (1 covariance on cross, 2 envelope on covariance; 0 = every wait matched;
 * a wait that gives up lets its workgroup go on, so the launch ends and its
 * results are not to be used).  reset != 0: clear the bits and re-zero the arrival
 * counters.  Returns DKG_OK (or a HIP error). */
int dkg_plan_status(const void* host_plan, int* err, int reset, void* stream);
/* 1 if dkg_plan_forward runs the plan's forward as the fused single launch, 0 if as the three stage kernels. */
int dkg_plan_fused(const void* host_plan);
/* Benchmark helper: average HIP-event duration (ms) of `reps` back-to-back
 * launches of one stage (0 cross_root, 1 posterior_cov, 2 envelope, 3 the
 * whole forward as dkg_plan_forward launches it) on
 * `stream`, after one full forward that primes its inputs; a final full
 * forward leaves kg / kg_pairs valid.  Synchronises. */
int dkg_plan_time_stage(const void* host_plan, const void* dev_plan, const double* xnew, int B, double* kg,
                        double* kg_pairs, void* stream, int stage, int reps, float* avg_ms);
/* As dkg_plan_time_stage for the launches of dkg_plan_forward_batches (nbatch batches of B candidates,
 * xnew [nbatch][B][d], kg [nbatch][B]): the stage as that entry launches it (stage 3: its three kernels). */
int dkg_plan_time_stage_batches(const void* host_plan, const void* dev_plan, const double* xnew, int B, int nbatch,
                                double* kg, void* stream, int stage, int reps, float* avg_ms);

/* Envelope stage alone: for P independent sets of L lines a_k + b_k z
 * (device, row-major [P][L]) kg[p] = E[max_k (a_k + b_k Z)] - max_k a_k, Z ~ N(0,1),
 * and optionally the number of upper-envelope lines n_hull[p] (nullable).
 * Replaces calculate_epigraph_indices + calculate_expected_value_of_piecewise_
 * linear_function + the baseline subtraction (discretekg.py:225-233, 341-452);
 * L = 0 -> DKG_ERR_NO_LINES (the reference's ValueError, :466-470).  Any L. */
int dkg_lines_kg(const double* intercepts, const double* slopes, int P, int L, double* kg, int* n_hull,
                 void* stream);

/* The reference's epigraph, exactly: calculate_epigraph_indices
 * (discretekg.py:341-412) for P sets of L lines (device, [P][L]).
 *   indices      : device int64 [P][cap], the envelope's line indices left to right
 *   intersections: device [P][cap - 1], the breakpoints between them (nullable if cap == 1)
 *   count        : device int [P], the envelope size m (entries beyond cap are not written)
 * Same walk as the reference: lines ordered by slope ascending then intercept
 * descending, each step to the later line of a different slope whose
 * intersection -(a_i - a_j)/(b_i - b_j) is first, ties to the first in that
 * order; the intersections are the same IEEE values.  Every |b| < 1e-9 -> the
 * first line of maximal intercept, no intersections (:363-367).  Among exact
 * duplicate lines (equal slope and intercept) the lowest index is returned
 * (the reference's first sort is not stable for more than 16 lines on CPU
 * torch; any duplicate is an equal line).  L = 0 -> DKG_ERR_NO_LINES. */
int dkg_epigraph(const double* intercepts, const double* slopes, int P, int L, int cap, long long* indices,
                 double* intersections, int* count, void* stream);

/* calculate_expected_value_of_piecewise_linear_function (discretekg.py:415-452)
 * for P functions of m pieces: out[p] = sum_j a_j (Phi(c_j) - Phi(c_{j-1}))
 * - b_j (phi(c_j) - phi(c_{j-1})), c_0 = -inf, c_m = +inf, boundaries [P][m-1]
 * (device; nullable when m == 1).  m = 0 -> DKG_ERR_NO_LINES. */
int dkg_pwl_expectation(const double* intercepts, const double* slopes, const double* boundaries, int P, int m,
                        double* out, void* stream);

/* The lines the plan's envelope stage builds for candidates xnew (device,
 * B x d): intercepts / slopes device [B][S][N + 1], line 0 the candidate
 * itself (discretekg.py:182-223 full, :300-321 decoupled), bit-identical to
 * the envelope's.  Runs the cross and covariance stages (an F32 plan: its fp32 contractions). */
int dkg_plan_lines(const void* host_plan, const void* dev_plan, const double* xnew, int B, double* intercepts,
                   double* slopes, void* stream);

/* Debug: per-workgroup phase stamps of the three forward kernels, written when
 * the env var DKG_DEBUG_STAMPS=1 at plan creation: [3][1024][8] words (slot 0
 * s_memrealtime at start, 1..6 s_memtime at phase boundaries, 7 s_memrealtime
 * at end); n words are copied. */
int dkg_debug_read_kstamps(unsigned long long* host, int n);

/* Debug/self-test of the register-only wave butterflies the kernels use
 * (DPP row ops + ds_bpermute for the 16/32 steps): in[64] -> out[512]; out[64 s + l] is the
 * partner value lane l receives at butterfly step s (0..5), out[384 + l] the
 * wave sum and out[448 + l] the wave max seen by lane l. */
int dkg_debug_wave_ops(const double* in, double* out, void* stream);

/* Debug/self-test: C[16x16] = A[16x4] B[4x16] (row-major, device) with one
 * v_mfma_f64_16x16x4_f64 using the operand/result lane maps the kernels assume. */
int dkg_debug_mfma_f64(const double* a, const double* b, double* c, void* stream);

/* The opt-in fp64 covariance block kernels for the launches that would take them (bits below; tests and A/B
 * measurements; initially from the environment variables DKG_COV_BLK / DKG_COV_REC2 / DKG_COV_REG).  Every one
 * gives the bits of the default kernels.  Returns the previous mask; a mask < 0 only reads it.
 * Process-wide: call it with no forward in flight. */
#define DKG_COV_ENABLE_BLK 1  /* 64 x 32 LDS-staged blocks, three workgroups per CU */
#define DKG_COV_ENABLE_REC2 2 /* m = 2, d <= 2: both outputs' whole records from one 8-wave workgroup per CU */
#define DKG_COV_ENABLE_REG 4  /* register-operand blocks, any m, one 8-wave workgroup per CU */
int dkg_debug_cov_kernels(int mask);

/* ---- Launcher: captured forward graphs of several streams enqueued side by side from host threads.
 * A hipGraphLaunch costs ~1 us of host time per kernel node plus ~9 us; one thread launching every
 * stream's graphs in turn leaves the last stream idle for the others' launches.  The
 * launcher keeps `threads - 1` worker threads (the caller is thread 0); stream s's graphs
 * graphs[offs[s] .. offs[s+1]) (hipGraphExec_t) are launched in order on streams[s] (hipStream_t) by
 * thread s % threads.  dkg_launcher_graphs returns once every launch call has returned; concurrent
 * calls on one launcher are serialised (a launcher runs one launch set at a time).  Armed
 * workers spin (wake-up in ~1 us) for `seconds`; otherwise they sleep on a condition variable.
 * Host-side scheduling only (the reference has no counterpart: its forward is a Python loop,
 * discretekg.py:145-159); no kernel is launched that the caller did not capture. */
int dkg_launcher_create(int threads, void** launcher);
int dkg_launcher_arm(void* launcher, double seconds);
int dkg_launcher_graphs(void* launcher, int n_streams, void* const* streams, const int* offs,
                        void* const* graphs);
int dkg_launcher_destroy(void* launcher);

#ifdef __cplusplus
}
#endif
#endif /* DKG_AMD_DKG_H */
