// Error reporting / version entry points of the C-ABI (include/comet_hip.h).
#include <string>

#include "../../include/comet_hip.h"

namespace comet {
static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }
}  // namespace comet

extern "C" int comet_version(void) { return 1; }
extern "C" const char* comet_last_error(void) { return comet::g_last_error.c_str(); }
