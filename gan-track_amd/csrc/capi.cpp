// ABI bookkeeping of libsg2hip: version and the per-thread last-error message.
#include <string>

#include "sg2_common.h"

namespace sg2 {
static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }
static thread_local bool g_acc_zeroed = false;
bool accumulators_prezeroed() { return g_acc_zeroed; }
static thread_local bool g_ws_clean = false;
bool workspace_clean() { return g_ws_clean; }
}  // namespace sg2

extern "C" void sg2_set_zeroed_accumulators(int on) { sg2::g_acc_zeroed = on != 0; }
extern "C" void sg2_set_clean_workspace(int on) { sg2::g_ws_clean = on != 0; }

extern "C" int sg2_abi_version(void) { return SG2_ABI_VERSION; }
extern "C" const char* sg2_last_error(void) { return sg2::g_last_error.c_str(); }
