// envelope_kernel instantiations for output bucket M = 8 (forward and gradient).
#include "dkg_device.h"

namespace dkg {

hipError_t launch_env_m8(bool grad, int lines, bool stream, const EnvLaunch& a) {
  return grad ? launch_env_bucket<8, true>(lines, stream, a) : launch_env_bucket<8, false>(lines, stream, a);
}

}  // namespace dkg
