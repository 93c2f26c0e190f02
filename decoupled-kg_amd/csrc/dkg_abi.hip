// C ABI of the Discrete-KG library (include/dkg.h).  Host-side validation,
// workspace carving and kernel sequencing; no device work happens here.
#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <string>

#include "dkg_kernels.h"

using namespace dkg;

namespace {

thread_local std::string g_err;
unsigned long long* g_kstamps_buf = nullptr;  // debug phase stamps (allocated on first use, kept)

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

}  // namespace

// dkg_kernels.h: the thread-local error message of the other host translation units (dkg_launch.hip)
int dkg::report_error(int code, const char* msg) {
  g_err = msg;
  return code;
}

namespace {

int hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) return fail(DKG_ERR_HIP, "%s: %s", what, hipGetErrorString(e));
  return DKG_OK;
}

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

struct WsLayout {
  size_t sync_bytes;  // the fused forward's counter block, at offset 0 (zeroed by one memset)
  size_t jq[DKG_MAX_OUTPUTS];
  size_t gmu[DKG_MAX_OUTPUTS];
  size_t qxrm[DKG_MAX_OUTPUTS];
  size_t qdrm[DKG_MAX_OUTPUTS];
  size_t q[DKG_MAX_OUTPUTS];
  size_t kx[DKG_MAX_OUTPUTS];  // 0: none (cross_kfill off for this output)
  size_t q32[DKG_MAX_OUTPUTS], root32[DKG_MAX_OUTPUTS], disc32[DKG_MAX_OUTPUTS];
  size_t kx32[DKG_MAX_OUTPUTS];  // 0: none (F32 plans with the K(x, X) fill only)
  size_t mux[DKG_MAX_OUTPUTS];
  size_t var[DKG_MAX_OUTPUTS];
  size_t mux_all, var_all, cov_all, mu_all;
  size_t wg_part;
  size_t wg_gpart;
  size_t tickets;
  size_t dup;
  size_t hull_pairs;
  size_t icpt, itop, itopk;  // 0: none (streaming envelope)
  size_t total;
};

static int max_np_of(const dkg_output* outs, int m) {
  int np = 0;
  for (int i = 0; i < m; ++i) np = std::max(np, pad16(outs[i].n));
  return np;
}

WsLayout layout(const dkg_output* outs, int m, int N, int B, int S, int d = 0, int flags = 0) {
  WsLayout L{};
  const size_t Bp = pad16(std::max(B, 1));
  // fused hand-off counters, one per 128-byte line: cnt1 [m][Bp / 16], cnt2 [ceil(B / 32)], done; then the err word
  L.sync_bytes = ((((size_t)m * (Bp / 16) + (Bp + 31) / 32 + 1) * HANDOFF_STRIDE * sizeof(unsigned long long) +
                   sizeof(int)) + 15) & ~(size_t)15;
  size_t off = align256(L.sync_bytes);
  for (int i = 0; i < m; ++i) {
    if (flags & DKG_PLAN_GRAD) {
      L.jq[i] = off;
      off = align256(off + (size_t)d * Bp * pad16(outs[i].n) * sizeof(double));
      L.gmu[i] = off;
      off = align256(off + (size_t)d * Bp * sizeof(double));
      L.qxrm[i] = off;
      off = align256(off + Bp * pad16(outs[i].n) * sizeof(double));
      L.qdrm[i] = off;
      off = align256(off + (size_t)std::max(N, 1) * pad16(outs[i].n) * sizeof(double));
    }
    L.q[i] = off;
    off = align256(off + Bp * pad16(outs[i].n) * sizeof(double));
    L.kx[i] = 0;
    if (cross_kfill_launch(max_np_of(outs, m), B)) {  // the launch covers every output of the plan
      L.kx[i] = off;
      off = align256(off + Bp * pad16(outs[i].n) * sizeof(double));
    }
    if (flags & DKG_PLAN_F32) {
      const size_t np = pad16(outs[i].n);
      L.q32[i] = off;
      off = align256(off + Bp * np * sizeof(float));
      L.root32[i] = off;
      off = align256(off + np * np * sizeof(float));
      L.disc32[i] = off;
      off = align256(off + (size_t)pad16(std::max(N, 1)) * np * sizeof(float));
      L.kx32[i] = 0;
      if (L.kx[i]) {
        L.kx32[i] = off;
        off = align256(off + Bp * np * sizeof(float));
      }
    }
  }
  // contiguous blocks (the envelope stage addresses them from kernel-argument
  // base pointers): means and variances at the candidates [m][Bp]; the
  // covariance rows [B][N][rec] and mu_D [N][rec] as line records
  // (rec = cov_rec(m) doubles per line, outputs side by side)
  const size_t rec = (size_t)cov_rec(m);
  L.mux_all = off;
  off = align256(off + (size_t)m * Bp * sizeof(double));
  L.var_all = off;
  off = align256(off + (size_t)m * Bp * sizeof(double));
  L.cov_all = off;
  off = align256(off + rec * std::max(B, 1) * std::max(N, 1) * sizeof(double));
  L.mu_all = off;
  off = align256(off + rec * std::max(N, 1) * sizeof(double));
  for (int i = 0; i < m; ++i) {
    L.mux[i] = L.mux_all + (size_t)i * Bp * sizeof(double);
    L.var[i] = L.var_all + (size_t)i * Bp * sizeof(double);
  }
  int sw, split;
  envelope_geometry(std::max(B, 1), std::max(S, 1), &sw, &split, !(flags & DKG_PLAN_FUSED));
  // split > 1: every pair's KG (and, value+gradient, its dKG/dx) for the last workgroup's ordered sums
  const size_t pcols = (size_t)std::max(S, 1) + pair_groups(std::max(S, 1));  // pair values + group terms
  L.wg_part = off;
  off = align256(off + (split > 1 ? (size_t)std::max(B, 1) * pcols * sizeof(double) : 0));
  L.wg_gpart = off;
  off = align256(off + ((flags & DKG_PLAN_GRAD) && split > 1 ? (size_t)std::max(B, 1) * pcols * d * sizeof(double) : 0));
  L.tickets = off;
  off = align256(off + Bp * (pair_groups(std::max(S, 1)) + 1) * sizeof(int));
  L.dup = off;
  off = align256(off + Bp * sizeof(int));
  L.hull_pairs = off;
  off = align256(off + (size_t)std::max(B, 1) * std::max(S, 1) * sizeof(int));
  if (N + 1 <= 64 * 33) {  // the staged forward's intercept cache (Plan::icpt)
    L.icpt = off;
    off = align256(off + (size_t)std::max(S, 1) * 64 * env_slots(N + 1) * sizeof(double));
    L.itop = off;
    off = align256(off + (size_t)std::max(S, 1) * sizeof(double));
    L.itopk = off;
    off = align256(off + (size_t)std::max(S, 1) * 2 * sizeof(int));
  }
  L.total = off;
  return L;
}

int check_outputs(const dkg_output* outs, int m, int d) {
  if (outs == nullptr) return fail(DKG_ERR_ARG, "outs is NULL");
  if (m < 1 || m > DKG_MAX_OUTPUTS) return fail(DKG_ERR_UNSUPPORTED, "m=%d outputs (supported 1..%d)", m, DKG_MAX_OUTPUTS);
  if (d < 1 || d > DKG_MAX_DIM) return fail(DKG_ERR_UNSUPPORTED, "d=%d (supported 1..%d)", d, DKG_MAX_DIM);
  for (int i = 0; i < m; ++i) {
    const dkg_output& o = outs[i];
    if (o.n < 1) return fail(DKG_ERR_ARG, "output %d: n=%d training points", i, o.n);
    if (pad16(o.n) > 1024) return fail(DKG_ERR_UNSUPPORTED, "output %d: n=%d > 1024 training points", i, o.n);
    if (cross_root_lds_bytes(pad16(o.n), d) > 160 * 1024)
      return fail(DKG_ERR_UNSUPPORTED, "output %d: n=%d, d=%d exceed the cross stage's LDS budget", i, o.n, d);
    if (o.kernel < DKG_MATERN12 || o.kernel > DKG_RBF) return fail(DKG_ERR_ARG, "output %d: kernel id %d", i, o.kernel);
    if (!o.inv_lengthscale || !o.train_x || !o.alpha || !o.root_frag)
      return fail(DKG_ERR_ARG, "output %d: missing device state pointer", i);
  }
  return DKG_OK;
}

int build_plan(const dkg_output* outs, int m, int d, const double* disc, int N, const double* weights, int S,
               int target, int max_B, void* workspace, size_t workspace_bytes, Plan* P, int flags = 0) {
  int st = check_outputs(outs, m, d);
  if (st) return st;
  if (max_B < 0 || N < 0) return fail(DKG_ERR_ARG, "negative size B=%d N=%d", max_B, N);
  if (S < 1) return fail(DKG_ERR_ARG, "S=%d scalarisations", S);
  if (target < -1 || target >= m) return fail(DKG_ERR_ARG, "target_output_ix=%d out of range for %d outputs", target, m);
  if (N > (1 << 22)) return fail(DKG_ERR_UNSUPPORTED, "N=%d discretisation points (supported <= %d)", N, 1 << 22);
  int sw, split;
  envelope_geometry(std::max(max_B, 1), S, &sw, &split, !(flags & DKG_PLAN_FUSED));
  int max_np = 16;
  for (int i = 0; i < m; ++i) max_np = std::max(max_np, pad16(outs[i].n));
  // the envelope stages the line data in LDS when it fits and the lines fit
  // the register slots; otherwise it streams them from global memory
  const bool want_grad = (flags & DKG_PLAN_GRAD) != 0;
  bool stream = N + 1 > 64 * 33 || envelope_lds_bytes(m, N, sw, S, false) > 160 * 1024 ||
                (want_grad && envelope_grad_lds_bytes(m, N, sw, S, d, max_np, false) > 160 * 1024);
  if (envelope_lds_bytes(m, N, sw, S, true) > 160 * 1024)
    return fail(DKG_ERR_UNSUPPORTED, "S=%d x m=%d weights exceed the envelope stage's LDS", S, m);
  if (!weights || !workspace || (N > 0 && !disc)) return fail(DKG_ERR_ARG, "NULL data pointer");
  for (int i = 0; i < m; ++i)
    if (N > 0 && (!outs[i].disc_frag || !outs[i].disc_mean))
      return fail(DKG_ERR_ARG, "output %d: discretisation caches missing", i);
  if (flags & ~(DKG_PLAN_GRAD | DKG_PLAN_FORCE_WALK | DKG_PLAN_F32 | DKG_PLAN_FUSED | DKG_PLAN_NO_CHAIN))
    return fail(DKG_ERR_ARG, "unknown plan flags 0x%x", flags);
  if (want_grad && (flags & DKG_PLAN_F32))
    return fail(DKG_ERR_UNSUPPORTED, "the fp32 plan (DKG_PLAN_F32) is forward only; the gradient runs in fp64");
  if (want_grad && envelope_grad_lds_bytes(m, N, sw, S, d, max_np, true) > 160 * 1024)
    return fail(DKG_ERR_UNSUPPORTED, "gradient: m=%d outputs, n=%d, d=%d exceed the envelope stage's LDS", m, max_np,
                d);
  const WsLayout L = layout(outs, m, N, max_B, S, d, flags);
  if (workspace_bytes < L.total)
    return fail(DKG_ERR_WORKSPACE, "workspace %zu bytes < required %zu", workspace_bytes, L.total);
  char* ws = static_cast<char*>(workspace);
  *P = Plan{};
  P->m = m;
  P->d = d;
  P->N = N;
  P->S = S;
  P->target = target;
  P->max_B = max_B;
  P->max_np = 16;
  P->sw = sw;
  P->split = split;
  P->disc = (N > 0) ? disc : reinterpret_cast<const double*>(ws);  // always a readable address
  P->weights = weights;
  P->grad = want_grad ? 1 : 0;
  P->f32 = (flags & DKG_PLAN_F32) ? 1 : 0;
  P->stream = stream ? 1 : 0;
  P->bpad = pad16(std::max(max_B, 1));
  for (int i = 0; i < m; ++i) {
    P->o[i] = outs[i];
    P->max_np = std::max(P->max_np, pad16(outs[i].n));
    if (P->grad) {
      P->jq[i] = reinterpret_cast<double*>(ws + L.jq[i]);
      P->gmu[i] = reinterpret_cast<double*>(ws + L.gmu[i]);
      P->qxrm[i] = reinterpret_cast<double*>(ws + L.qxrm[i]);
      P->qdrm[i] = reinterpret_cast<double*>(ws + L.qdrm[i]);
    }
    P->q[i] = reinterpret_cast<double*>(ws + L.q[i]);
    P->kx[i] = L.kx[i] ? reinterpret_cast<double*>(ws + L.kx[i]) : nullptr;
    if (flags & DKG_PLAN_F32) {
      P->q32[i] = reinterpret_cast<float*>(ws + L.q32[i]);
      P->root32[i] = reinterpret_cast<float*>(ws + L.root32[i]);
      P->disc32[i] = reinterpret_cast<float*>(ws + L.disc32[i]);
      P->kx32[i] = L.kx32[i] ? reinterpret_cast<float*>(ws + L.kx32[i]) : nullptr;
    }
    P->mux[i] = reinterpret_cast<double*>(ws + L.mux[i]);
    P->var[i] = reinterpret_cast<double*>(ws + L.var[i]);
  }
  P->mux_all = reinterpret_cast<double*>(ws + L.mux_all);
  P->var_all = reinterpret_cast<double*>(ws + L.var_all);
  P->cov_all = reinterpret_cast<double*>(ws + L.cov_all);
  P->mu_all = reinterpret_cast<double*>(ws + L.mu_all);
  P->cov_stride = (int64_t)std::max(N, 1) * cov_rec(m);
  P->wg_part = reinterpret_cast<double*>(ws + L.wg_part);
  P->tickets = reinterpret_cast<int*>(ws + L.tickets);
  P->dup = reinterpret_cast<int*>(ws + L.dup);
  P->wg_gpart = reinterpret_cast<double*>(ws + L.wg_gpart);
  P->hull_pairs = reinterpret_cast<int*>(ws + L.hull_pairs);
  // the intercept cache serves the staged forward envelope (a gradient plan's forward included)
  if (L.icpt && !stream) {
    P->icpt = reinterpret_cast<double*>(ws + L.icpt);
    P->icpt_stride = 64 * env_slots(N + 1);
    P->itop = reinterpret_cast<double*>(ws + L.itop);
    P->itopk = reinterpret_cast<int*>(ws + L.itopk);
  }
  static const char* denv = std::getenv("DKG_DEBUG_ENV_FLAGS");
  static const char* dcov = std::getenv("DKG_DEBUG_COV_FLAGS");
  P->debug_env = (denv ? std::atoi(denv) : 0) | ((flags & DKG_PLAN_FORCE_WALK) ? 1 : 0) |
                  ((flags & DKG_PLAN_NO_CHAIN) ? 8 : 0);
  P->debug_cov = dcov ? std::atoi(dcov) : 0;
  static const char* dst = std::getenv("DKG_DEBUG_STAMPS");
  P->debug_stamp = dst ? std::atoi(dst) : 0;
  // the fused one-launch forward (dkg_fused.h) only on explicit request (DKG_PLAN_FUSED): fp64, staged
  // lines, no test hooks; its bounded in-launch waits report give-ups through dkg_plan_status
  const bool split_stages = !(flags & DKG_PLAN_FUSED) || (flags & DKG_PLAN_FORCE_WALK);
  P->sync = reinterpret_cast<unsigned long long*>(ws);
  P->sync_bytes = L.sync_bytes;
  {
    const size_t words = ((size_t)m * (pad16(std::max(max_B, 1)) / 16) + (pad16(std::max(max_B, 1)) + 31) / 32 + 1) *
                         HANDOFF_STRIDE;
    P->sync_err = reinterpret_cast<int*>(ws + words * sizeof(unsigned long long));
  }
  P->fused = (!split_stages && !P->f32 && !P->stream && N >= 1 && N + 1 <= 64 * 17 && !P->debug_env && !P->debug_cov &&
              !DKG_ABLATIONS && fused_lds_bytes_host(*P) <= 160 * 1024)
                 ? 1
                 : 0;
  if (P->debug_stamp) {
    if (!g_kstamps_buf &&
        hip_check(hipMalloc(&g_kstamps_buf, sizeof(unsigned long long) * 3 * KST_WG * 8), "hipMalloc(stamps)"))
      return DKG_ERR_HIP;
    P->kstamps = g_kstamps_buf;
  }
  return DKG_OK;
}

int run_forward(const Plan& h, const Plan* dev, const double* xnew, int B, double* kg, double* kg_pairs,
                hipStream_t stream, float* stage_ms) {
  if (B < 0) return fail(DKG_ERR_ARG, "negative B=%d", B);
  if (B == 0) return DKG_OK;
  if (B > h.max_B) return fail(DKG_ERR_ARG, "B=%d candidates > plan capacity %d", B, h.max_B);
  if (!xnew || !kg) return fail(DKG_ERR_ARG, "NULL data pointer");
  hipEvent_t ev[4];
  int st;
  if (stage_ms)
    for (int k = 0; k < 4; ++k)
      if ((st = hip_check(hipEventCreate(&ev[k]), "hipEventCreate"))) return st;
  if ((st = hip_check(stage_ms ? launch_forward(h, dev, xnew, B, kg, kg_pairs, stream, ev)
                                : launch_forward_auto(h, dev, xnew, B, kg, kg_pairs, stream),
                      "forward")))
    return st;
  if (stage_ms) {
    if ((st = hip_check(hipEventSynchronize(ev[3]), "hipEventSynchronize"))) return st;
    for (int k = 0; k < 3; ++k) (void)hipEventElapsedTime(&stage_ms[k], ev[k], ev[k + 1]);
    for (int k = 0; k < 4; ++k) (void)hipEventDestroy(ev[k]);
  }
  return DKG_OK;
}

size_t plan_slot_bytes() { return align256(sizeof(Plan)); }

// mu_D of every output into the plan's line records [N][cov_rec(m)] (stream
// ordered); the padding components (m < cov_rec(m)) of mu_D and of every
// covariance row are zeroed here once (the covariance stage writes components
// < m only), so they enter the line build as 0 with a zero weight.
int copy_disc_means(const Plan& P, hipStream_t s) {
  if (int st = hip_check(hipMemsetAsync(P.sync, 0, P.sync_bytes, s), "hipMemsetAsync(sync)")) return st;
  const int rec = cov_rec(P.m);
  if (rec > P.m && P.N > 0) {
    const size_t rows = (size_t)std::max(P.max_B, 1) * P.N;
    int st = hip_check(hipMemsetAsync(P.mu_all, 0, sizeof(double) * rec * P.N, s), "hipMemsetAsync(mu_D)");
    if (!st) st = hip_check(hipMemsetAsync(P.cov_all, 0, sizeof(double) * rec * rows, s), "hipMemsetAsync(cov)");
    if (st) return st;
  }
  for (int i = 0; i < P.m && P.f32; ++i) {
    // F32: fp32 copies of R^T and Q_D for the fp32 contractions
    int st = hip_check(launch_frag_to_f32(P.o[i].root_frag, P.o[i].n, P.o[i].n, P.root32[i], s), "frag_to_f32(R)");
    if (st) return st;
    if (P.N > 0 &&
        (st = hip_check(launch_frag_to_f32(P.o[i].disc_frag, P.N, P.o[i].n, P.disc32[i], s), "frag_to_f32(Q_D)")))
      return st;
  }
  for (int i = 0; i < P.m && P.N > 0; ++i) {
    int st = hip_check(hipMemcpy2DAsync(P.mu_all + i, sizeof(double) * rec, P.o[i].disc_mean, sizeof(double),
                                        sizeof(double), P.N, hipMemcpyDeviceToDevice, s), "hipMemcpy2DAsync(mu_D)");
    if (st) return st;
    // GRAD: row-major Q_D for the envelope's per-line row gathers
    if (P.grad && (st = hip_check(launch_unpack_rows(P.o[i].disc_frag, P.N, P.o[i].n, P.qdrm[i], s), "unpack_rows")))
      return st;
  }
  if (P.icpt) return hip_check(launch_intercepts(P, s), "intercepts");
  return DKG_OK;
}

// One-shot path: plan built on the host per call, its device copy placed in
// the workspace tail (one small host-to-device copy per call).
int forward_oneshot(const dkg_output* outs, int m, int d, const double* disc, int N, const double* xnew, int B,
                    const double* weights, int S, int target, double* kg, double* kg_pairs, void* workspace,
                    size_t workspace_bytes, hipStream_t stream, float* stage_ms) {
  if (B == 0) return check_outputs(outs, m, d);
  const size_t slot = plan_slot_bytes() + 256;
  const size_t avail = workspace_bytes > slot ? workspace_bytes - slot : 0;
  thread_local Plan h;
  int st = build_plan(outs, m, d, disc, N, weights, S, target, B, workspace, avail, &h);
  if (st) return st;
  if ((st = copy_disc_means(h, stream))) return st;
  Plan* dev = reinterpret_cast<Plan*>((reinterpret_cast<uintptr_t>(workspace) + avail + 255) & ~(uintptr_t)255);
  if ((st = hip_check(hipMemcpyAsync(dev, &h, sizeof(Plan), hipMemcpyHostToDevice, stream), "hipMemcpyAsync")))
    return st;
  return run_forward(h, dev, xnew, B, kg, kg_pairs, stream, stage_ms);
}

}  // namespace

extern "C" {

int dkg_abi_version(void) { return DKG_ABI_VERSION; }

const char* dkg_last_error(void) { return g_err.c_str(); }

size_t dkg_frag_elems(int rows, int n) { return (size_t)pad16(std::max(rows, 0)) * pad16(std::max(n, 0)); }

size_t dkg_prepare_workspace(int n) {
  if (n < 1) return 0;
  return align256((size_t)n * n * sizeof(double)) + 256;
}

// Argument checks of one output's preparation (dkg_prepare_output / dkg_prepare_outputs).
static int check_prepare(const dkg_output* o, int d, const double* train_y, int max_tries, const double* L,
                         const void* work, size_t work_bytes, const double* alpha, const double* root_frag) {
  if (!o || !train_y || !L || !work || !alpha || !root_frag || !o->inv_lengthscale || !o->train_x)
    return fail(DKG_ERR_ARG, "NULL pointer");
  const int n = o->n;
  if (n < 1) return fail(DKG_ERR_ARG, "n=%d training points", n);
  if (pad16(n) > 1024) return fail(DKG_ERR_UNSUPPORTED, "n=%d > 1024 training points", n);
  if (d < 1 || d > DKG_MAX_DIM) return fail(DKG_ERR_UNSUPPORTED, "d=%d (supported 1..%d)", d, DKG_MAX_DIM);
  if (o->kernel < DKG_MATERN12 || o->kernel > DKG_RBF) return fail(DKG_ERR_ARG, "kernel id %d", o->kernel);
  if (max_tries < 0) return fail(DKG_ERR_ARG, "max_tries=%d", max_tries);
  if (work_bytes < dkg_prepare_workspace(n))
    return fail(DKG_ERR_WORKSPACE, "workspace %zu bytes < required %zu", work_bytes, dkg_prepare_workspace(n));
  return DKG_OK;
}

static int* prepare_info(void* work, int n) {
  return reinterpret_cast<int*>(static_cast<char*>(work) + align256((size_t)n * n * sizeof(double)));
}

// psd_safe_cholesky's attempts first .. max_tries of one output (attempt 0: no jitter; then absolute jitter
// 1e-8 * 10^(attempt - 1)), each checked on the host.  *jit: the jitter that worked.
static int cholesky_attempts(const dkg_output* o, int d, double* L, double* X, int* info, int first, int max_tries,
                             hipStream_t s, double* jit) {
  int st, h_info = 1;
  for (int attempt = first; attempt <= max_tries; ++attempt) {
    *jit = attempt == 0 ? 0.0 : 1e-8 * std::pow(10.0, attempt - 1);
    if ((st = hip_check(launch_kernel_matrix(*o, d, o->train_x, o->n, o->train_x, o->n, o->noise + *jit, L, s),
                        "kernel_matrix")))
      return st;
    if ((st = hip_check(hipMemsetAsync(info, 0, sizeof(int), s), "hipMemsetAsync")) ||
        (st = hip_check(launch_cholesky(L, X, o->n, info, s), "cholesky")) ||
        (st = hip_check(hipMemcpyAsync(&h_info, info, sizeof(int), hipMemcpyDeviceToHost, s), "hipMemcpyAsync")) ||
        (st = hip_check(hipStreamSynchronize(s), "hipStreamSynchronize")))
      return st;
    if (h_info == 0) return DKG_OK;
  }
  return fail(DKG_ERR_NOT_PD, "covariance not positive definite after %d jitter retries (pivot %d)", max_tries,
              h_info);
}

int dkg_prepare_output(const dkg_output* o, int d, const double* train_y, int max_tries, double* L, void* work,
                       size_t work_bytes, double* alpha, double* root_frag, double* jitter_used, void* stream) {
  int st = check_prepare(o, d, train_y, max_tries, L, work, work_bytes, alpha, root_frag);
  if (st) return st;
  hipStream_t s = (hipStream_t)stream;
  const int n = o->n;
  double* X = static_cast<double*>(work);
  int* info = prepare_info(work, n);
  double jit = 0.0;
  if ((st = cholesky_attempts(o, d, L, X, info, 0, max_tries, s, &jit))) return st;
  if (jitter_used) *jitter_used = jit;
  if ((st = hip_check(launch_tri_inverse(L, X, n, info, s), "tri_inverse")) ||
      (st = hip_check(launch_alpha(X, train_y, o->mean_constant, n, alpha, info, s), "alpha")) ||
      (st = hip_check(launch_pack_linv(X, n, root_frag, s), "pack_linv")))
    return st;
  return DKG_OK;
}

int dkg_prepare_outputs(const dkg_output* outs, int m, int d, const double* const* train_y, int max_tries,
                        double* const* L, void* const* work, const size_t* work_bytes, double* const* alpha,
                        double* const* root_frag, double* jitter_used, void* stream) {
  if (!outs || m < 1 || m > DKG_MAX_OUTPUTS) return fail(DKG_ERR_ARG, "m=%d outputs (1..%d)", m, DKG_MAX_OUTPUTS);
  if (!train_y || !L || !work || !work_bytes || !alpha || !root_frag) return fail(DKG_ERR_ARG, "NULL pointer");
  int st;
  for (int i = 0; i < m; ++i)
    if ((st = check_prepare(&outs[i], d, train_y[i], max_tries, L[i], work[i], work_bytes[i], alpha[i], root_frag[i])))
      return st;
  hipStream_t s = (hipStream_t)stream;
  PrepBatch b{};
  int h_info[DKG_MAX_OUTPUTS];
  double jit[DKG_MAX_OUTPUTS];
  for (int i = 0; i < m; ++i) {
    b.A[i] = L[i];
    b.X[i] = static_cast<double*>(work[i]);
    b.n[i] = outs[i].n;
    b.info[i] = prepare_info(work[i], outs[i].n);
    jit[i] = 0.0;
    if ((st = hip_check(launch_kernel_matrix(outs[i], d, outs[i].train_x, outs[i].n, outs[i].train_x, outs[i].n,
                                             outs[i].noise, L[i], s), "kernel_matrix")) ||
        (st = hip_check(hipMemsetAsync(b.info[i], 0, sizeof(int), s), "hipMemsetAsync")))
      return st;
  }
  // every output's first attempt in one chain of launches, one status check for all
  if ((st = hip_check(launch_cholesky_batch(b, m, s), "cholesky_batch"))) return st;
  for (int i = 0; i < m; ++i)
    if ((st = hip_check(hipMemcpyAsync(&h_info[i], b.info[i], sizeof(int), hipMemcpyDeviceToHost, s),
                        "hipMemcpyAsync")))
      return st;
  if ((st = hip_check(hipStreamSynchronize(s), "hipStreamSynchronize"))) return st;
  for (int i = 0; i < m; ++i)  // the outputs that need jitter are retried on their own, as dkg_prepare_output
    if (h_info[i] != 0 &&
        (st = cholesky_attempts(&outs[i], d, L[i], b.X[i], b.info[i], 1, max_tries, s, &jit[i])))
      return st;
  if ((st = hip_check(launch_tri_inverse_batch(b, m, s), "tri_inverse_batch"))) return st;
  for (int i = 0; i < m; ++i) {
    if ((st = hip_check(launch_alpha(b.X[i], train_y[i], outs[i].mean_constant, outs[i].n, alpha[i], b.info[i], s),
                        "alpha")) ||
        (st = hip_check(launch_pack_linv(b.X[i], outs[i].n, root_frag[i], s), "pack_linv")))
      return st;
    if (jitter_used) jitter_used[i] = jit[i];
  }
  return DKG_OK;
}

int dkg_kernel_matrix(const dkg_output* o, int d, const double* x1, int n1, const double* x2, int n2,
                      double diag_add, double* out, void* stream) {
  if (!o || !x1 || !x2 || !out || !o->inv_lengthscale) return fail(DKG_ERR_ARG, "NULL pointer");
  if (d < 1 || d > DKG_MAX_DIM) return fail(DKG_ERR_UNSUPPORTED, "d=%d", d);
  if (n1 < 0 || n2 < 0) return fail(DKG_ERR_ARG, "negative size");
  if (n1 == 0 || n2 == 0) return DKG_OK;
  return hip_check(launch_kernel_matrix(*o, d, x1, n1, x2, n2, diag_add, out, (hipStream_t)stream),
                   "kernel_matrix_kernel");
}

int dkg_pack_root(const double* r, int n, double* root_frag, void* stream) {
  if (!r || !root_frag || n < 1) return fail(DKG_ERR_ARG, "bad arguments");
  return hip_check(launch_pack_root(r, n, root_frag, (hipStream_t)stream), "pack_root_kernel");
}

int dkg_cross_root(const dkg_output* o, int d, const double* x, int rows, double* q_frag, double* mean,
                   void* stream) {
  int st = check_outputs(o, 1, d);
  if (st) return st;
  if (rows < 0 || !q_frag || (rows > 0 && !x)) return fail(DKG_ERR_ARG, "bad arguments");
  if (rows == 0) return DKG_OK;
  CrossArgs ca{};
  ca.o = *o;
  ca.d = d;
  ca.rows = rows;
  ca.x = x;
  ca.q = q_frag;
  ca.mean = mean;
  return hip_check(launch_cross_root(ca, (hipStream_t)stream), "cross_root_kernel");
}

size_t dkg_forward_workspace(const dkg_output* outs, int m, int N, int B, int S) {
  if (!outs || m < 1 || m > DKG_MAX_OUTPUTS) return 0;
  return layout(outs, m, N, B, S).total + plan_slot_bytes() + 256;
}

int dkg_forward(const dkg_output* outs, int m, int d, const double* disc, int N, const double* xnew, int B,
                const double* weights, int S, int target, double* kg, double* kg_pairs, void* workspace,
                size_t workspace_bytes, void* stream) {
  return forward_oneshot(outs, m, d, disc, N, xnew, B, weights, S, target, kg, kg_pairs, workspace, workspace_bytes,
                         (hipStream_t)stream, nullptr);
}

int dkg_forward_timed(const dkg_output* outs, int m, int d, const double* disc, int N, const double* xnew,
                      int B, const double* weights, int S, int target, double* kg, double* kg_pairs,
                      void* workspace, size_t workspace_bytes, void* stream, float* stage_ms) {
  if (!stage_ms) return fail(DKG_ERR_ARG, "stage_ms is NULL");
  return forward_oneshot(outs, m, d, disc, N, xnew, B, weights, S, target, kg, kg_pairs, workspace, workspace_bytes,
                         (hipStream_t)stream, stage_ms);
}

size_t dkg_plan_bytes(void) { return sizeof(Plan); }

static int time_stage(const void* host_plan, const void* dev_plan, const double* xnew, int B, double* kg,
                      double* kg_pairs, void* stream, int stage, int reps, float* avg_ms, int geom_B) {
  if (!host_plan || !dev_plan || !avg_ms) return fail(DKG_ERR_ARG, "NULL pointer");
  if (stage < 0 || stage > 3 || reps < 1) return fail(DKG_ERR_ARG, "stage=%d reps=%d", stage, reps);
  const Plan& h = *static_cast<const Plan*>(host_plan);
  if (B < 1 || B > h.max_B) return fail(DKG_ERR_ARG, "B=%d outside [1, %d]", B, h.max_B);
  if (!xnew || !kg) return fail(DKG_ERR_ARG, "NULL data pointer");
  const Plan* dev = static_cast<const Plan*>(dev_plan);
  hipStream_t s = (hipStream_t)stream;
  hipEvent_t ev[2];
  int st;
  for (int k = 0; k < 2; ++k)
    if ((st = hip_check(hipEventCreate(&ev[k]), "hipEventCreate"))) return st;
  // prime the inputs of the timed stage, then time reps back-to-back launches of it alone
  if ((st = hip_check(launch_forward(h, dev, xnew, B, kg, kg_pairs, s, nullptr, geom_B), "forward"))) return st;
  (void)hipEventRecord(ev[0], s);
  for (int r = 0; r < reps; ++r)
    if ((st = hip_check(stage == 3 ? (geom_B ? launch_forward(h, dev, xnew, B, kg, nullptr, s, nullptr, geom_B)
                                             : launch_forward_auto(h, dev, xnew, B, kg, nullptr, s))
                                   : launch_stage(h, dev, xnew, B, kg, kg_pairs, s, stage, geom_B),
                        "stage")))
      return st;
  (void)hipEventRecord(ev[1], s);
  if ((st = hip_check(hipEventSynchronize(ev[1]), "hipEventSynchronize"))) return st;
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, ev[0], ev[1]);
  *avg_ms = ms / reps;
  for (int k = 0; k < 2; ++k) (void)hipEventDestroy(ev[k]);
  // leave kg / kg_pairs valid again (repeated stages accumulate into kg)
  return hip_check(launch_forward(h, dev, xnew, B, kg, kg_pairs, s, nullptr, geom_B), "forward");
}

int dkg_plan_time_stage(const void* host_plan, const void* dev_plan, const double* xnew, int B, double* kg,
                        double* kg_pairs, void* stream, int stage, int reps, float* avg_ms) {
  return time_stage(host_plan, dev_plan, xnew, B, kg, kg_pairs, stream, stage, reps, avg_ms, 0);
}

int dkg_plan_time_stage_batches(const void* host_plan, const void* dev_plan, const double* xnew, int B, int nbatch,
                                double* kg, void* stream, int stage, int reps, float* avg_ms) {
  if (B < 1 || nbatch < 1) return fail(DKG_ERR_ARG, "B=%d nbatch=%d", B, nbatch);
  if (!host_plan) return fail(DKG_ERR_ARG, "NULL plan pointer");
  // (as dkg_plan_forward_batches: the product in 64 bits, so a wrapped int cannot pass the capacity check)
  if ((long long)B * nbatch > static_cast<const Plan*>(host_plan)->max_B)
    return fail(DKG_ERR_ARG, "%d batches of B=%d candidates > plan capacity %d", nbatch, B,
                static_cast<const Plan*>(host_plan)->max_B);
  return time_stage(host_plan, dev_plan, xnew, B * nbatch, kg, nullptr, stream, stage, reps, avg_ms, B);
}

size_t dkg_plan_workspace(const dkg_output* outs, int m, int d, int N, int max_B, int S, int flags) {
  if (!outs || m < 1 || m > DKG_MAX_OUTPUTS) return 0;
  return layout(outs, m, N, max_B, S, d, flags).total;
}

int dkg_plan_init(const dkg_output* outs, int m, int d, const double* disc, int N, const double* weights, int S,
                  int target, int max_B, int flags, void* workspace, size_t workspace_bytes, void* host_plan,
                  void* dev_plan, void* stream) {
  if (!host_plan || !dev_plan) return fail(DKG_ERR_ARG, "NULL plan pointer");
  Plan* h = static_cast<Plan*>(host_plan);
  int st = build_plan(outs, m, d, disc, N, weights, S, target, max_B, workspace, workspace_bytes, h, flags);
  if (st) return st;
  if ((st = copy_disc_means(*h, (hipStream_t)stream))) return st;
  return hip_check(hipMemcpyAsync(dev_plan, h, sizeof(Plan), hipMemcpyHostToDevice, (hipStream_t)stream),
                   "hipMemcpyAsync");
}

int dkg_plan_forward(const void* host_plan, const void* dev_plan, const double* xnew, int B, double* kg,
                     double* kg_pairs, void* stream) {
  if (!host_plan || !dev_plan) return fail(DKG_ERR_ARG, "NULL plan pointer");
  return run_forward(*static_cast<const Plan*>(host_plan), static_cast<const Plan*>(dev_plan), xnew, B, kg, kg_pairs,
                     (hipStream_t)stream, nullptr);
}

int dkg_plan_forward_batches(const void* host_plan, const void* dev_plan, const double* xnew, int B, int nbatch,
                             double* kg, void* stream) {
  if (!host_plan || !dev_plan) return fail(DKG_ERR_ARG, "NULL plan pointer");
  const Plan& h = *static_cast<const Plan*>(host_plan);
  if (B < 0 || nbatch < 0) return fail(DKG_ERR_ARG, "negative size B=%d nbatch=%d", B, nbatch);
  if ((long long)B * nbatch == 0) return DKG_OK;
  if ((long long)B * nbatch > h.max_B)
    return fail(DKG_ERR_ARG, "%d batches x B=%d candidates > plan capacity %d", nbatch, B, h.max_B);
  if (!xnew || !kg) return fail(DKG_ERR_ARG, "NULL data pointer");
  // the three stage kernels over all nbatch * B candidates, the covariance blocks chosen for one batch of B
  return hip_check(launch_forward(h, static_cast<const Plan*>(dev_plan), xnew, B * nbatch, kg, nullptr,
                                  (hipStream_t)stream, nullptr, B),
                   "forward_batches");
}

int dkg_plan_forward_timed(const void* host_plan, const void* dev_plan, const double* xnew, int B, double* kg,
                           double* kg_pairs, void* stream, float* stage_ms) {
  if (!host_plan || !dev_plan || !stage_ms) return fail(DKG_ERR_ARG, "NULL pointer");
  return run_forward(*static_cast<const Plan*>(host_plan), static_cast<const Plan*>(dev_plan), xnew, B, kg, kg_pairs,
                     (hipStream_t)stream, stage_ms);
}

int dkg_plan_forward_grad(const void* host_plan, const void* dev_plan, const double* xnew, int B, double* kg,
                          double* dkg_dx, void* stream) {
  if (!host_plan || !dev_plan) return fail(DKG_ERR_ARG, "NULL plan pointer");
  const Plan& h = *static_cast<const Plan*>(host_plan);
  if (!h.grad) return fail(DKG_ERR_ARG, "plan was not initialised with DKG_PLAN_GRAD");
  if (B < 0) return fail(DKG_ERR_ARG, "negative B=%d", B);
  if (B == 0) return DKG_OK;
  if (B > h.max_B) return fail(DKG_ERR_ARG, "B=%d candidates > plan capacity %d", B, h.max_B);
  if (!xnew || !kg || !dkg_dx) return fail(DKG_ERR_ARG, "NULL data pointer");
  return hip_check(launch_forward_grad(h, static_cast<const Plan*>(dev_plan), xnew, B, kg, dkg_dx,
                                       (hipStream_t)stream), "forward_grad");
}

int dkg_plan_forward_grad_hostx(const void* host_plan, const void* dev_plan, const double* x_host, double* x_dev,
                                int B, double* kg, double* dkg_dx, double* out_host, void* stream) {
  if (!host_plan || !dev_plan) return fail(DKG_ERR_ARG, "NULL plan pointer");
  const Plan& h = *static_cast<const Plan*>(host_plan);
  if (!h.grad) return fail(DKG_ERR_ARG, "plan was not initialised with DKG_PLAN_GRAD");
  if (B < 0) return fail(DKG_ERR_ARG, "negative B=%d", B);
  if (B == 0) return DKG_OK;
  if (B > h.max_B) return fail(DKG_ERR_ARG, "B=%d candidates > plan capacity %d", B, h.max_B);
  if ((long long)B * h.d > DKG_XARG_MAX)
    return fail(DKG_ERR_ARG, "B*d=%lld > DKG_XARG_MAX=%d (use dkg_plan_forward_grad)", (long long)B * h.d, DKG_XARG_MAX);
  if (!x_host || !x_dev || !kg || !dkg_dx) return fail(DKG_ERR_ARG, "NULL data pointer");
  XArg xa;
  xa.n = B * h.d;
  for (int i = 0; i < xa.n; ++i) xa.v[i] = x_host[i];
  int st = hip_check(launch_forward_grad(h, static_cast<const Plan*>(dev_plan), x_dev, B, kg, dkg_dx,
                                         (hipStream_t)stream, &xa, out_host),
                     "forward_grad_hostx");
  if (st || !out_host) return st;
  return hip_check(hipStreamSynchronize((hipStream_t)stream), "hipStreamSynchronize");  // out_host is filled
}

int dkg_plan_status(const void* host_plan, int* err, int reset, void* stream) {
  if (!host_plan || !err) return fail(DKG_ERR_ARG, "NULL pointer");
  const Plan& h = *static_cast<const Plan*>(host_plan);
  hipStream_t s = (hipStream_t)stream;
  int st;
  if ((st = hip_check(hipMemcpyAsync(err, h.sync_err, sizeof(int), hipMemcpyDeviceToHost, s), "hipMemcpyAsync(err)")) ||
      (st = hip_check(hipStreamSynchronize(s), "hipStreamSynchronize")))
    return st;
  if (reset) return hip_check(hipMemsetAsync(h.sync, 0, h.sync_bytes, s), "hipMemsetAsync(sync)");
  return DKG_OK;
}

int dkg_plan_fused(const void* host_plan) { return host_plan ? static_cast<const Plan*>(host_plan)->fused : 0; }

int dkg_plan_hull_sizes(const void* host_plan, int* out, int B, void* stream) {
  if (!host_plan || !out) return fail(DKG_ERR_ARG, "NULL pointer");
  const Plan& h = *static_cast<const Plan*>(host_plan);
  if (B < 0 || B > h.max_B) return fail(DKG_ERR_ARG, "B=%d outside [0, %d]", B, h.max_B);
  if (B == 0) return DKG_OK;
  return hip_check(hipMemcpyAsync(out, h.hull_pairs, sizeof(int) * (size_t)B * h.S, hipMemcpyDeviceToDevice,
                                  (hipStream_t)stream), "hipMemcpyAsync(hull sizes)");
}

int dkg_lines_kg(const double* intercepts, const double* slopes, int P, int L, double* kg, int* n_hull,
                 void* stream) {
  if (P < 0 || L < 0) return fail(DKG_ERR_ARG, "negative size P=%d L=%d", P, L);
  if (P == 0) return DKG_OK;
  if (L == 0)
    return fail(DKG_ERR_NO_LINES, "Expected inputs to specify at least one line. Got intercepts.shape[-1]=0.");
  if (!intercepts || !slopes || !kg) return fail(DKG_ERR_ARG, "NULL pointer");
  return hip_check(launch_lines_kg(intercepts, slopes, P, L, kg, n_hull, nullptr, nullptr, 0, (hipStream_t)stream),
                   "lines_kg_kernel");
}

int dkg_epigraph(const double* intercepts, const double* slopes, int P, int L, int cap, long long* indices,
                 double* intersections, int* count, void* stream) {
  if (P < 0 || L < 0 || cap < 1) return fail(DKG_ERR_ARG, "bad size P=%d L=%d cap=%d", P, L, cap);
  if (P == 0) return DKG_OK;
  if (L == 0)
    return fail(DKG_ERR_NO_LINES, "Expected inputs to specify at least one line. Got intercepts.shape[-1]=0.");
  if (!intercepts || !slopes || !indices || !count || (cap > 1 && !intersections))
    return fail(DKG_ERR_ARG, "NULL pointer");
  return hip_check(launch_lines_kg(intercepts, slopes, P, L, nullptr, count, indices, intersections, cap,
                                   (hipStream_t)stream), "lines_kg_kernel(epigraph)");
}

int dkg_pwl_expectation(const double* intercepts, const double* slopes, const double* boundaries, int P, int m,
                        double* out, void* stream) {
  if (P < 0 || m < 0) return fail(DKG_ERR_ARG, "negative size P=%d m=%d", P, m);
  if (P == 0) return DKG_OK;
  if (m == 0)
    return fail(DKG_ERR_NO_LINES, "Expected inputs to specify at least one line. Got intercepts.shape[-1]=0.");
  if (!intercepts || !slopes || !out || (m > 1 && !boundaries)) return fail(DKG_ERR_ARG, "NULL pointer");
  return hip_check(launch_pwl_expectation(intercepts, slopes, boundaries, P, m, out, (hipStream_t)stream),
                   "pwl_expectation_kernel");
}

int dkg_plan_lines(const void* host_plan, const void* dev_plan, const double* xnew, int B, double* intercepts,
                   double* slopes, void* stream) {
  if (!host_plan || !dev_plan) return fail(DKG_ERR_ARG, "NULL plan pointer");
  const Plan& h = *static_cast<const Plan*>(host_plan);
  if (B < 0 || B > h.max_B) return fail(DKG_ERR_ARG, "B=%d outside [0, %d]", B, h.max_B);
  if (B == 0) return DKG_OK;
  if (!xnew || !intercepts || !slopes) return fail(DKG_ERR_ARG, "NULL data pointer");
  // (an F32 plan exports the lines its fp32 contractions give: the error model's check, tools/f32_debug.py)
  const Plan* dev = static_cast<const Plan*>(dev_plan);
  hipStream_t s = (hipStream_t)stream;
  int st;
  for (int stage = 0; stage < 2; ++stage)  // K(x, X) R, means; covariance rows, variances (kg is only zeroed)
    if ((st = hip_check(launch_stage(h, dev, xnew, B, intercepts, nullptr, s, stage), "stage"))) return st;
  return hip_check(launch_lines_export(h, dev, B, intercepts, slopes, s), "lines_export_kernel");
}

int dkg_debug_read_kstamps(unsigned long long* host, int n) {
  if (!host || n < 0) return fail(DKG_ERR_ARG, "bad arguments");
  if (!g_kstamps_buf) return fail(DKG_ERR_ARG, "no plan was built with DKG_DEBUG_STAMPS=1");
  const size_t words = std::min<size_t>((size_t)n, (size_t)3 * KST_WG * 8);
  return hip_check(hipMemcpy(host, g_kstamps_buf, words * sizeof(unsigned long long), hipMemcpyDeviceToHost),
                   "hipMemcpy(stamps)");
}

int dkg_debug_cov_kernels(int mask) {
  if (mask < 0) {
    const int cur = set_cov_enabled(0);
    set_cov_enabled(cur);
    return cur;
  }
  return set_cov_enabled(mask);
}

int dkg_debug_wave_ops(const double* in, double* out, void* stream) {
  if (!in || !out) return fail(DKG_ERR_ARG, "NULL pointer");
  return hip_check(launch_debug_wave(in, out, (hipStream_t)stream), "debug_wave_kernel");
}

int dkg_debug_mfma_f64(const double* a, const double* b, double* c, void* stream) {
  if (!a || !b || !c) return fail(DKG_ERR_ARG, "NULL pointer");
  return hip_check(launch_debug_mfma(a, b, c, (hipStream_t)stream), "debug_mfma_kernel");
}

}  // extern "C"
