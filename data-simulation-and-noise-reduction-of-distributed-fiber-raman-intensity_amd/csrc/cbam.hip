// ADSDN / APIDN forward (CBAM networks): implemented in a later revision.
#include "common.hpp"

namespace rdn {

size_t cbam_workspace_bytes(int, int, int64_t, int64_t) { return 0; }

hipError_t launch_cbam_forward(int, int, const uint8_t*, const float*, float*, int64_t, int, void*, size_t,
                               hipStream_t) {
  return hipErrorNotSupported;
}

}  // namespace rdn
