// ABI bookkeeping of libsg2hip: version and the per-thread last-error message.
#include <cstdlib>
#include <string>

#include "sg2_common.h"

namespace sg2 {
static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }
static thread_local bool g_acc_zeroed = false;
bool accumulators_prezeroed() { return g_acc_zeroed; }
static thread_local bool g_ws_clean = false;
bool workspace_clean() { return g_ws_clean; }
bool det_assign_on() {
    static const bool on = [] { const char* e = getenv("SG2_DET_ASSIGN"); return !(e && e[0] == '0'); }();
    return on;
}
// Process-wide, not per thread: autograd runs the backward passes of a deterministic scope on its own device
// thread, whose calls must see the mode (sg2_set_deterministic is called between launches, never concurrently).
static float* g_det_base = nullptr;
static int64_t g_det_cap = 0;
bool det_on() { return g_det_base != nullptr; }
DetArena::DetArena() : base_(g_det_base), cap_(g_det_cap), off_(0) {}
float* DetArena::get(int64_t n) {
    const int64_t a = (n + 63) & ~(int64_t)63;   // 256-byte aligned slices
    if (!base_ || off_ + a > cap_) return nullptr;
    float* p = base_ + off_;
    off_ += a;
    return p;
}
}  // namespace sg2

extern "C" void sg2_set_deterministic(void* scratch, int64_t bytes) {
    sg2::g_det_base = (scratch && bytes > 0) ? static_cast<float*>(scratch) : nullptr;
    sg2::g_det_cap = sg2::g_det_base ? bytes / (int64_t)sizeof(float) : 0;
}

extern "C" void sg2_set_zeroed_accumulators(int on) { sg2::g_acc_zeroed = on != 0; }
extern "C" void sg2_set_clean_workspace(int on) { sg2::g_ws_clean = on != 0; }

extern "C" int sg2_abi_version(void) { return SG2_ABI_VERSION; }
extern "C" const char* sg2_last_error(void) { return sg2::g_last_error.c_str(); }
