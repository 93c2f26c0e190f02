// envelope_kernel instantiations for output bucket M = 3 (forward and gradient), and the fused
// one-launch forward of the same bucket (dkg_fused.h).
#include "dkg_fused.h"

namespace dkg {

hipError_t launch_env_m3(bool grad, int lines, bool stream, const EnvLaunch& a) {
  return grad ? launch_env_bucket<3, true>(lines, stream, a) : launch_env_bucket<3, false>(lines, stream, a);
}

hipError_t launch_fused_m3(int dim_b, int lines, const FusedArgs& a, size_t lds, hipStream_t s) {
  return launch_fused_bucket<3>(dim_b, lines, a, lds, s);
}

}  // namespace dkg
