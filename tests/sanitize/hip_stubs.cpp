// hip_stubs.cpp — the device-side helpers libapg's host sources call, for the
// host-only sanitizer build (tests/sanitize/Makefile links no HIP kernels).
// The drivers never reach them (no GPU here); they fail loudly if they do.
#include <string>

#include "../../allpathslg_amd/csrc/apg_core.hpp"

namespace apg {
int dreads_device_shape(apg_ctx*, apg_dreads*, const uint64_t*, bool, const char* who) {
  set_error(std::string(who) + ": device read sets need the HIP build (sanitizer build has no kernels)");
  return APG_E_UNSUPPORTED;
}
}  // namespace apg
