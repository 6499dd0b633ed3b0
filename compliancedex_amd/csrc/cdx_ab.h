// Run-time A/B switches of the native library.  The shipped libcdx.so reads NONE of them: ab_env() returns null
// unless the library is built with -DCDX_AB_SWITCHES (the A/B builds of tools/, `build_device(defines=...)`), so a
// variable left in a user's environment can neither switch off the screened closure's audit and repair
// (CDX_SCREEN_AUDIT, CDX_SCREEN_REPAIR) nor change its schedule.  cdx_ab_switches() reports the build's choice.
// The two path switches whose results the test suite checks bit for bit against the default (CDX_KABSCH_AHEAD,
// CDX_VAR_LATE: tests/test_screen.py) stay readable in every build.
#pragma once
#include <cstdlib>

namespace cdx {
inline const char* ab_env(const char* name) {
#if defined(CDX_AB_SWITCHES)
  return getenv(name);
#else
  (void)name;
  return nullptr;
#endif
}
}  // namespace cdx
