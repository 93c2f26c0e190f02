// Kernel argument blocks and launch helpers shared by the kernels TU and the C ABI TU.
#pragma once

#include "dkg_common.h"

namespace dkg {

struct CrossArgs {
  Outputs outs;
  int d;
  int rows;
  const double* x;                       // [rows x d]
  double* q[DKG_MAX_OUTPUTS];            // fragment-packed Q per output
  double* mean[DKG_MAX_OUTPUTS];         // [pad16(rows)] per output (nullable)
  int* tickets;                          // zeroed by one workgroup (nullable)
  int n_tickets;
};

struct CovArgs {
  Outputs outs;
  int d, N, B;
  const double* xnew;                    // [B x d]
  const double* disc;                    // [N x d]
  const double* q[DKG_MAX_OUTPUTS];      // fragment-packed Q_x per output
  double* cov[DKG_MAX_OUTPUTS];          // [B x N] per output
};

struct EnvArgs {
  Outputs outs;
  int m, N, S, B, target;
  const double* weights;                 // [S x m]
  const double* q[DKG_MAX_OUTPUTS];
  const double* mux[DKG_MAX_OUTPUTS];
  const double* cov[DKG_MAX_OUTPUTS];
  double* kg;                            // [B]
  double* pairs_out;                     // [B x S] nullable
  double* wg_part;                       // [B x SPLIT]
  int* tickets;                          // [B], zero on entry
};

hipError_t launch_kernel_matrix(const dkg_output& o, int d, const double* x1, int n1, const double* x2, int n2,
                                double diag_add, double* out, hipStream_t s);
hipError_t launch_pack_root(const double* r, int n, double* rf, hipStream_t s);
hipError_t launch_cross_root(const CrossArgs& a, int m, int max_np, hipStream_t s);
hipError_t launch_posterior_cov(const CovArgs& a, int m, hipStream_t s);
hipError_t launch_envelope(const EnvArgs& a, int waves_per_wg, int split, hipStream_t s);
hipError_t launch_lines_kg(const double* a, const double* b, int P, int L, double* kg, int* nhull, hipStream_t s);
hipError_t launch_debug_mfma(const double* a, const double* b, double* c, hipStream_t s);

// Launch geometry of the envelope stage for (B, S): waves per workgroup and
// workgroups per candidate.
void envelope_geometry(int B, int S, int* waves_per_wg, int* split);

}  // namespace dkg
