// envelope_kernel instantiations for output bucket M = 4 (forward and gradient).
#include "dkg_device.h"

namespace dkg {

hipError_t launch_env_m4(bool grad, int lines, bool stream, const EnvLaunch& a) {
  return grad ? launch_env_bucket<4, true>(lines, stream, a) : launch_env_bucket<4, false>(lines, stream, a);
}

}  // namespace dkg
