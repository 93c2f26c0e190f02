// C ABI of the Discrete-KG library (include/dkg.h).  Host-side validation,
// workspace carving and kernel sequencing; no device work happens here.
#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <string>

#include "dkg_kernels.h"

using namespace dkg;

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

int hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) return fail(DKG_ERR_HIP, "%s: %s", what, hipGetErrorString(e));
  return DKG_OK;
}

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

struct WsLayout {
  size_t q[DKG_MAX_OUTPUTS];
  size_t mux[DKG_MAX_OUTPUTS];
  size_t cov[DKG_MAX_OUTPUTS];
  size_t wg_part;
  size_t tickets;
  size_t total;
};

WsLayout layout(const dkg_output* outs, int m, int N, int B, int S) {
  WsLayout L{};
  size_t off = 0;
  const size_t Bp = pad16(std::max(B, 1));
  for (int i = 0; i < m; ++i) {
    L.q[i] = off;
    off = align256(off + Bp * pad16(outs[i].n) * sizeof(double));
    L.mux[i] = off;
    off = align256(off + Bp * sizeof(double));
    L.cov[i] = off;
    off = align256(off + (size_t)std::max(B, 1) * std::max(N, 1) * sizeof(double));
  }
  int sw, split;
  envelope_geometry(std::max(B, 1), std::max(S, 1), &sw, &split);
  L.wg_part = off;
  off = align256(off + (size_t)std::max(B, 1) * split * sizeof(double));
  L.tickets = off;
  off = align256(off + Bp * sizeof(int));
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
    if (o.kernel < DKG_MATERN12 || o.kernel > DKG_RBF) return fail(DKG_ERR_ARG, "output %d: kernel id %d", i, o.kernel);
    if (!o.inv_lengthscale || !o.train_x || !o.alpha || !o.root_frag)
      return fail(DKG_ERR_ARG, "output %d: missing device state pointer", i);
  }
  return DKG_OK;
}

int forward_impl(const dkg_output* outs, int m, int d, const double* disc, int N, const double* xnew, int B,
                 const double* weights, int S, int target, double* kg, double* kg_pairs, void* workspace,
                 size_t workspace_bytes, hipStream_t stream, float* stage_ms) {
  int st = check_outputs(outs, m, d);
  if (st) return st;
  if (B < 0 || N < 0) return fail(DKG_ERR_ARG, "negative size B=%d N=%d", B, N);
  if (S < 1) return fail(DKG_ERR_ARG, "S=%d scalarisations", S);
  if (target < -1 || target >= m) return fail(DKG_ERR_ARG, "target_output_ix=%d out of range for %d outputs", target, m);
  if (N + 1 > 64 * 33) return fail(DKG_ERR_UNSUPPORTED, "N=%d discretisation points (supported <= %d)", N, 64 * 33 - 1);
  if (B == 0) return DKG_OK;
  if (!xnew || !weights || !kg || !workspace || (N > 0 && !disc)) return fail(DKG_ERR_ARG, "NULL data pointer");
  for (int i = 0; i < m; ++i)
    if (N > 0 && (!outs[i].disc_frag || !outs[i].disc_mean))
      return fail(DKG_ERR_ARG, "output %d: discretisation caches missing", i);
  const WsLayout L = layout(outs, m, N, B, S);
  if (workspace_bytes < L.total)
    return fail(DKG_ERR_WORKSPACE, "workspace %zu bytes < required %zu", workspace_bytes, L.total);
  char* ws = static_cast<char*>(workspace);

  Outputs O{};
  int max_np = 16;
  for (int i = 0; i < m; ++i) {
    O.o[i] = outs[i];
    max_np = std::max(max_np, pad16(outs[i].n));
  }

  hipEvent_t ev[4];
  if (stage_ms) {
    for (int k = 0; k < 4; ++k)
      if ((st = hip_check(hipEventCreate(&ev[k]), "hipEventCreate"))) return st;
    (void)hipEventRecord(ev[0], stream);
  }

  CrossArgs ca{};
  ca.outs = O;
  ca.d = d;
  ca.rows = B;
  ca.x = xnew;
  for (int i = 0; i < m; ++i) {
    ca.q[i] = reinterpret_cast<double*>(ws + L.q[i]);
    ca.mean[i] = reinterpret_cast<double*>(ws + L.mux[i]);
  }
  ca.tickets = reinterpret_cast<int*>(ws + L.tickets);
  ca.n_tickets = B;
  if ((st = hip_check(launch_cross_root(ca, m, max_np, stream), "cross_root_kernel"))) return st;
  if (stage_ms) (void)hipEventRecord(ev[1], stream);

  CovArgs cv{};
  cv.outs = O;
  cv.d = d;
  cv.N = N;
  cv.B = B;
  cv.xnew = xnew;
  cv.disc = disc;
  for (int i = 0; i < m; ++i) {
    cv.q[i] = ca.q[i];
    cv.cov[i] = reinterpret_cast<double*>(ws + L.cov[i]);
  }
  if (N > 0)
    if ((st = hip_check(launch_posterior_cov(cv, m, stream), "posterior_cov_kernel"))) return st;
  if (stage_ms) (void)hipEventRecord(ev[2], stream);

  EnvArgs ea{};
  ea.outs = O;
  ea.m = m;
  ea.N = N;
  ea.S = S;
  ea.B = B;
  ea.target = target;
  ea.weights = weights;
  for (int i = 0; i < m; ++i) {
    ea.q[i] = ca.q[i];
    ea.mux[i] = ca.mean[i];
    ea.cov[i] = cv.cov[i];
  }
  ea.kg = kg;
  ea.pairs_out = kg_pairs;
  ea.wg_part = reinterpret_cast<double*>(ws + L.wg_part);
  ea.tickets = ca.tickets;
  int sw, split;
  envelope_geometry(B, S, &sw, &split);
  if ((st = hip_check(launch_envelope(ea, sw, split, stream), "envelope_kernel"))) return st;

  if (stage_ms) {
    (void)hipEventRecord(ev[3], stream);
    if ((st = hip_check(hipEventSynchronize(ev[3]), "hipEventSynchronize"))) return st;
    for (int k = 0; k < 3; ++k) (void)hipEventElapsedTime(&stage_ms[k], ev[k], ev[k + 1]);
    for (int k = 0; k < 4; ++k) (void)hipEventDestroy(ev[k]);
  }
  return DKG_OK;
}

}  // namespace

extern "C" {

int dkg_abi_version(void) { return DKG_ABI_VERSION; }

const char* dkg_last_error(void) { return g_err.c_str(); }

size_t dkg_frag_elems(int rows, int n) { return (size_t)pad16(std::max(rows, 0)) * pad16(std::max(n, 0)); }

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
  ca.outs.o[0] = *o;
  ca.d = d;
  ca.rows = rows;
  ca.x = x;
  ca.q[0] = q_frag;
  ca.mean[0] = mean;
  return hip_check(launch_cross_root(ca, 1, pad16(o->n), (hipStream_t)stream), "cross_root_kernel");
}

size_t dkg_forward_workspace(const dkg_output* outs, int m, int N, int B, int S) {
  if (!outs || m < 1 || m > DKG_MAX_OUTPUTS) return 0;
  return layout(outs, m, N, B, S).total;
}

int dkg_forward(const dkg_output* outs, int m, int d, const double* disc, int N, const double* xnew, int B,
                const double* weights, int S, int target, double* kg, double* kg_pairs, void* workspace,
                size_t workspace_bytes, void* stream) {
  return forward_impl(outs, m, d, disc, N, xnew, B, weights, S, target, kg, kg_pairs, workspace,
                      workspace_bytes, (hipStream_t)stream, nullptr);
}

int dkg_forward_timed(const dkg_output* outs, int m, int d, const double* disc, int N, const double* xnew,
                      int B, const double* weights, int S, int target, double* kg, double* kg_pairs,
                      void* workspace, size_t workspace_bytes, void* stream, float* stage_ms) {
  if (!stage_ms) return fail(DKG_ERR_ARG, "stage_ms is NULL");
  return forward_impl(outs, m, d, disc, N, xnew, B, weights, S, target, kg, kg_pairs, workspace,
                      workspace_bytes, (hipStream_t)stream, stage_ms);
}

int dkg_lines_kg(const double* intercepts, const double* slopes, int P, int L, double* kg, int* n_hull,
                 void* stream) {
  if (P < 0 || L < 0) return fail(DKG_ERR_ARG, "negative size P=%d L=%d", P, L);
  if (P == 0) return DKG_OK;
  if (L == 0)
    return fail(DKG_ERR_NO_LINES, "Expected inputs to specify at least one line. Got intercepts.shape[-1]=0.");
  if (L > 64 * 33) return fail(DKG_ERR_UNSUPPORTED, "L=%d lines per set (supported <= %d)", L, 64 * 33);
  if (!intercepts || !slopes || !kg) return fail(DKG_ERR_ARG, "NULL pointer");
  return hip_check(launch_lines_kg(intercepts, slopes, P, L, kg, n_hull, (hipStream_t)stream), "lines_kg_kernel");
}

int dkg_debug_mfma_f64(const double* a, const double* b, double* c, void* stream) {
  if (!a || !b || !c) return fail(DKG_ERR_ARG, "NULL pointer");
  return hip_check(launch_debug_mfma(a, b, c, (hipStream_t)stream), "debug_mfma_kernel");
}

}  // extern "C"
