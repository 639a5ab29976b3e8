// capi.hip — error state and version of the libreidmi C ABI (include/reidmi.h).
#include "common.h"

namespace reidmi {
static thread_local std::string g_err;
void set_error(const std::string& m) { g_err = m; }
int fail(int code, const std::string& m) {
    g_err = m;
    return code;
}
}  // namespace reidmi

REIDMI_API const char* reidmi_last_error(void) { return reidmi::g_err.c_str(); }
// 2: per-call GEMM tiling / distance variant entry points replace the process-global setters;
//    RCCL exchange (reidmi_comm_*); re-ranking without capacity limits.
REIDMI_API int reidmi_abi_version(void) { return 3; }
