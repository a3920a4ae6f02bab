// ABI bookkeeping of libsg2hip: version and the per-thread last-error message.
#include <string>

#include "sg2_common.h"

namespace sg2 {
static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }
}  // namespace sg2

extern "C" int sg2_abi_version(void) { return SG2_ABI_VERSION; }
extern "C" const char* sg2_last_error(void) { return sg2::g_last_error.c_str(); }
