// Error reporting / version entry points of the C-ABI (include/comet_hip.h).
#include <string>

#include "../../include/comet_hip.h"

#include <cstdio>

namespace comet {
static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }
#ifdef COMET_DEBUG
static int g_dbg_host = 0;  // OR of every assertion word read so far (comet_debug_flags)
void debug_record(const char* name, int word) {
  g_dbg_host |= word;
  char buf[64];
  snprintf(buf, sizeof buf, " (assertion word 0x%08x)", word);
  set_error(std::string(name) + ": device-side index check failed" + buf);
}
#endif
}  // namespace comet

extern "C" int comet_debug_flags(int clear) {
#ifdef COMET_DEBUG
  const int w = comet::g_dbg_host;
  if (clear) comet::g_dbg_host = 0;
  return w;
#else
  (void)clear;
  return -1;
#endif
}

extern "C" int comet_version(void) { return 1; }
extern "C" const char* comet_last_error(void) { return comet::g_last_error.c_str(); }
