// Kernel argument blocks and launch helpers shared by the kernels TU and the C ABI TU.
#pragma once

#include "dkg_common.h"

namespace dkg {

// Line records: the posterior means mu_D and a candidate's covariance row are
// kept [N][cov_rec(m)] (all outputs of a line side by side, zero-padded to a
// power of two), in global memory and staged as is, so a lane reads two
// outputs of a line with one 16-byte ds_read_b128 (256 B/clk) instead of
// per-output 8-byte reads the compiler pairs into ds_read2st64_b64 (128 B/clk).
__host__ __device__ constexpr int cov_rec(int m) { return m <= 1 ? 1 : m <= 2 ? 2 : m <= 4 ? 4 : 8; }

// Groups of 8 scalarisation pairs: the envelope stage's fixed summation order (envelope_body).
__host__ __device__ constexpr int pair_groups(int S) { return (S + 7) >> 3; }
// Plan::dup: no discretisation point coincides with the candidate.
constexpr int DUP_NONE = 0x7fffffff;

// Stage ablations (empty cross / covariance / envelope launches selected by
// DKG_DEBUG_COV_FLAGS 2 / 1 and DKG_DEBUG_ENV_FLAGS 2; cross_big_kernel's means alone / Q_X blocks alone by
// DKG_DEBUG_COV_FLAGS 16 / 32) exist only in builds
// with -DDKG_ABLATIONS=1: the check is a dependent scalar load at kernel entry.
#ifndef DKG_ABLATIONS
#define DKG_ABLATIONS 0
#endif

// Everything a forward needs besides the candidates, resident in device memory
// (written once per (model, discretisation, weights) by dkg_plan_init): the
// kernels take a pointer to it, so each launch carries ~40 bytes of arguments
// instead of a ~1 KiB by-value block (measured ~1.5 us of launch cost).
// Large n: K(x, X) is filled once per forward by its own kernel (cross_kfill_kernel) and the cross
// workgroups load their slab of it.  Every column-pair group of a row tile otherwise evaluates the
// kernel over the columns its wider tile needs: at n = 1024 (64 tiles, 32 groups) each entry ~24 times,
// which took most of the stage.  At the headline's n = 256 the extra launch costs more than it saves
// (profiles/r02/r02zz).
#ifndef DKG_CROSS_KFILL
#define DKG_CROSS_KFILL 1
#endif
__host__ __device__ inline bool cross_kfill(int np) { return DKG_CROSS_KFILL && np >= 512; }
// Launches over many candidates (a launch of several forward batches, dkg_plan_forward_batches) fill K(x, X)
// once with the separate kernel at any n: the fill replicated over the column-pair groups of a row tile (~4.5x
// at n = 256) is then work the whole device waits on, not latency one forward hides.  Same bits either way.
#ifndef DKG_KFILL_MIN_B
#define DKG_KFILL_MIN_B 512
#endif
constexpr int KFILL_MIN_B = DKG_KFILL_MIN_B;
__host__ __device__ inline bool cross_kfill_launch(int np, int B) {
  return DKG_CROSS_KFILL && (np >= 512 || B >= KFILL_MIN_B);
}

// Register slots per lane for a staged (non-streaming) line set of `lines`
// lines: the envelope_kernel instantiation launch_env_bucket picks.
__host__ __device__ inline int env_slots(int lines) {
  return lines <= 64 * 2 ? 2 : lines <= 64 * 8 ? 8 : lines <= 64 * 17 ? 17 : 33;
}

struct Plan {
  dkg_output o[DKG_MAX_OUTPUTS];
  int32_t m, d, N, S, target;       // target < 0: all outputs observed
  int32_t max_B, max_np;            // workspace sized for max_B candidates; max n_pad over outputs
  int32_t sw, split;                // envelope geometry: waves per workgroup, workgroups per candidate
  int32_t debug_env, debug_cov;     // test / ablation switches (0 in production)
  int32_t debug_stamp;              // 1: per-workgroup phase stamps into g_kstamps (0 in production)
  int32_t grad;                     // workspace holds the gradient buffers (DKG_PLAN_GRAD)
  int32_t bpad;                     // pad16(max_B): rows of the fragment-packed candidate buffers
  int32_t stream;                   // envelope streams the lines from global memory (large N)
  int32_t f32;                      // DKG_PLAN_F32: fp32 contractions (q32 / root32 / disc32)
  const double* disc;               // [N x d]
  const double* weights;            // [S x m]
  double* q[DKG_MAX_OUTPUTS];       // fragment-packed K(x, X) R per output (workspace)
  double* kx[DKG_MAX_OUTPUTS];      // large n (cross_kfill): K(x, X) per output in the cross stage's B-operand
                                    // order [B_pad / 16][n_pad / 4][64], filled once per forward (else null)
  double* mux[DKG_MAX_OUTPUTS];     // posterior mean at the candidates per output (workspace)
  double* var[DKG_MAX_OUTPUTS];     // noiseless posterior variance s - |Q_X[b]|^2 per output (workspace)
  double* jq[DKG_MAX_OUTPUTS];      // GRAD: J_g = dK(x,X)/dx_g R, row-major [d][bpad][n_pad] per output
  double* qxrm[DKG_MAX_OUTPUTS];    // GRAD: Q_X = K(x,X) R row-major [bpad][n_pad] per output
  double* qdrm[DKG_MAX_OUTPUTS];    // GRAD: Q_D = K(D,X) R row-major [N][n_pad] per output (written at plan init)
  double* gmu[DKG_MAX_OUTPUTS];     // GRAD: [d][bpad] model-space mean gradients
  unsigned long long* kstamps;      // debug_stamp: [3][KST_WG][8] phase stamps (device)
  double* mux_all;                  // [m][bpad]  = mux[0..m)
  double* var_all;                  // [m][bpad]  = var[0..m)
  double* cov_all;                  // [max_B][N][cov_rec(m)] posterior covariance rows, line records (workspace)
  double* mu_all;                   // [N][cov_rec(m)] the outputs' disc_mean, line records
  int64_t cov_stride;               // N * cov_rec(m): doubles per candidate in cov_all
  double* wg_part;                  // [B][S + ng] pair values, then group terms (ng = ceil(S / 8); split > 1 only)
  int* tickets;                     // [B][ng + 1] group and candidate arrival counters (zeroed by the cross stage)
  // [B]: the lowest record k with z_k == x_b exactly (DUP_NONE: none), from the covariance stage (r^2 = 0).
  // The reference's joint posterior over [x_b; D] makes line 0 and line k + 1 exact copies there (same rows
  // of one covariance matrix), and the walk then takes line 0 (lowest index) while torch.max splits the
  // gradient of max a between them; the envelope builds line 0 from record k so it is the same copy.
  int* dup;
  double* wg_gpart;                 // GRAD: [B][S + ng][d] as wg_part, for dKG/dx (split > 1 only)
  float* q32[DKG_MAX_OUTPUTS];      // F32: quad-packed K(x, X) R per output (workspace)
  float* root32[DKG_MAX_OUTPUTS];   // F32: quad-packed R^T (fp32 copy of root_frag, plan init)
  float* disc32[DKG_MAX_OUTPUTS];   // F32: quad-packed Q_D (fp32 copy of disc_frag, plan init)
  int* hull_pairs;                  // [max_B x S] upper-envelope lines per pair (written with kg_pairs)
  int32_t fused;                    // dkg_plan_forward runs the fused one-launch forward (dkg_fused.h)
  unsigned long long* sync;         // fused hand-off counters: cnt1 [m][rt], cnt2 [nrb], done (zeroed)
  int* sync_err;                    // fused waits that gave up (bits), after the counters
  size_t sync_bytes;                // bytes of the counter block (sync .. sync_err), a multiple of 16
  // Staged forward: the intercepts of lines k >= 1 depend on the weights and mu_D only, not on the
  // candidates -- a_k = a_off + sum_i w_i sd_i mu_i(z_k), discretekg.py:201-213 -- so the plan keeps them
  // (dkg_plan_init, the envelope's own arithmetic: bit-identical lines) beside each scalarisation's largest.
  double* icpt;                     // [S][icpt_stride]: slot k = a_k for 1 <= k <= N, NaN at k = 0 and k > N
  int32_t icpt_stride;              // 64 * env_slots(N + 1): one entry per register slot of the envelope
  double* itop;                     // [S]: max_{k >= 1} a_k (-inf when N = 0)
  int* itopk;                       // [S][2]: the first k >= 1 attaining it, and how many lines do
  float* kx32[DKG_MAX_OUTPUTS];     // F32 with the K(x, X) fill: kx's entries quad-packed in fp32 (frag32_index),
                                    // the B operand of cross_big32_kernel (kx itself still feeds the fp64 means)
};

// By-value arguments of the state-preparation use of the cross stage.
struct CrossArgs {
  dkg_output o;
  int d, rows;
  const double* x;  // [rows x d]
  double* q;        // fragment-packed Q
  double* mean;     // [pad16(rows)] (nullable)
};

hipError_t launch_kernel_matrix(const dkg_output& o, int d, const double* x1, int n1, const double* x2, int n2,
                                double diag_add, double* out, hipStream_t s);
hipError_t launch_pack_root(const double* r, int n, double* rf, hipStream_t s);
// State preparation (dkg_linalg.hip): blocked Cholesky with device status (L in A's lower triangle, the
// inverses of its diagonal blocks in X's), triangular inverse X = L^{-1}, alpha = Linv^T Linv (y - c),
// root_frag from Linv.
hipError_t launch_cholesky(double* A, double* X, int n, int* info, hipStream_t s);
// Several outputs' factorisations side by side: every launch of the blocked chains carries all of them
// (blockIdx.y = output).  A = the matrix (Cholesky: L on return) , X = the inverse (diagonal blocks written
// by the Cholesky, the rest by the inverse).
struct PrepBatch {
  double* A[DKG_MAX_OUTPUTS];
  double* X[DKG_MAX_OUTPUTS];
  int n[DKG_MAX_OUTPUTS];
  int* info[DKG_MAX_OUTPUTS];
};
hipError_t launch_cholesky_batch(const PrepBatch& b, int m, hipStream_t s);
hipError_t launch_tri_inverse_batch(const PrepBatch& b, int m, hipStream_t s);
hipError_t launch_tri_inverse(double* L, double* X, int n, const int* info, hipStream_t s);
hipError_t launch_alpha(const double* X, const double* y, double c, int n, double* alpha, const int* info,
                        hipStream_t s);
hipError_t launch_pack_linv(const double* X, int n, double* rf, hipStream_t s);
// fp32 quad-packed copy (frag32_index) of a pair-packed fp64 (rows x n) matrix.
hipError_t launch_frag_to_f32(const double* frag, int rows, int n, float* out, hipStream_t s);
// The plan's per-scalarisation intercepts and their maxima (Plan::icpt / itop / itopk), from mu_all.
hipError_t launch_intercepts(const Plan& h, hipStream_t s);
// Row-major copy [rows][n_pad] of a fragment-packed (rows x n) matrix.
hipError_t launch_unpack_rows(const double* frag, int rows, int n, double* out, hipStream_t s);
hipError_t launch_cross_root(const CrossArgs& a, hipStream_t s);
// Value and gradient: kg[B] and dkg[B x d] (d KG(x_b) / d x_b), plan built with DKG_PLAN_GRAD.
// Candidates by value in the first kernel's arguments (dkg_plan_forward_grad_hostx); n = 0: unused.
struct XArg {
  double v[DKG_XARG_MAX];
  int n;
};
// hout (nullable): pinned host [kg (B) | dkg (B x d)] written by the envelope stage itself (split <= 2).
hipError_t launch_forward_grad(const Plan& h, const Plan* dev, const double* xnew, int B, double* kg, double* dkg,
                               hipStream_t s, const XArg* xa = nullptr, double* hout = nullptr);
size_t envelope_grad_lds_bytes(int m, int N, int waves, int S, int d, int max_np, bool stream);
// One stage of the forward (0 cross_root, 1 posterior_cov, 2 envelope) on stream s.  geom_B (0: B) is the
// batch size the covariance block shape is chosen for: a launch over K batches of geom_B candidates
// (dkg_plan_forward_batches) takes the blocks of one geom_B forward, so its results are those of K forwards.
hipError_t launch_stage(const Plan& h, const Plan* dev, const double* xnew, int B, double* kg, double* pairs,
                        hipStream_t s, int stage, int geom_B = 0);
hipError_t launch_forward(const Plan& host, const Plan* dev, const double* xnew, int B, double* kg, double* pairs,
                          hipStream_t s, hipEvent_t* ev, int geom_B = 0);
// The fused one-launch forward (dkg_fused.h) when the plan allows it (Plan::fused, no kg_pairs);
// otherwise the three stage kernels.  Same bits.
// Dynamic LDS bytes of the fused forward for a plan (dkg_fused.h fused_lds_bytes).
size_t fused_lds_bytes_host(const Plan& h);
// Sets dkg_last_error()'s thread-local message (host translation units other than dkg_abi.hip); returns code.
int report_error(int code, const char* msg);
hipError_t launch_forward_auto(const Plan& host, const Plan* dev, const double* xnew, int B, double* kg,
                               double* pairs, hipStream_t s);
// Envelope stage alone over P sets of L lines: KG, envelope sizes (nullable) and, when idx is given, the
// reference walk's indices [P][cap] and intersections [P][cap - 1] (lines_kg_kernel / lines_walk_kernel).
hipError_t launch_lines_kg(const double* a, const double* b, int P, int L, double* kg, int* nhull, long long* idx,
                           double* xs, int cap, hipStream_t s);
// The lines of every (candidate, scalarisation) pair after stages 0-1 (dkg_plan_lines).
hipError_t launch_lines_export(const Plan& h, const Plan* dev, int B, double* a_out, double* b_out, hipStream_t s);
// Reference formula of E[f(Z)] for P piecewise-linear f of m pieces (dkg_pwl_expectation).
hipError_t launch_pwl_expectation(const double* a, const double* b, const double* c, int P, int m, double* out,
                                  hipStream_t s);
// Per-workgroup phase stamps of the forward kernels: [3 kernels][KST_WG][8].
constexpr int KST_WG = 1024;
hipError_t launch_debug_wave(const double* in, double* out, hipStream_t s);
// The opt-in fp64 covariance block kernels (dkg_debug_cov_kernels): sets the mask, returns the previous one.
int set_cov_enabled(int mask);
hipError_t launch_debug_mfma(const double* a, const double* b, double* c, hipStream_t s);

// Launch geometry of the envelope stage for (B, S): waves per workgroup and
// workgroups per candidate.
void envelope_geometry(int B, int S, int* waves_per_wg, int* split, bool narrow);
// mu: the mu_D records are staged too (the gradient and fused envelopes; the staged forward reads the plan's
// intercept cache instead)
size_t envelope_lds_bytes(int m, int N, int waves, int S, bool stream, bool grad = false, bool mu = true);
size_t cross_root_lds_bytes(int np, int d);

}  // namespace dkg
