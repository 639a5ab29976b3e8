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
// 3: RCCL exchange (reidmi_comm_*); re-ranking without capacity limits;
// 4: the forced-variant entry points moved to libreidmi_tools.so (include/reidmi_tools.h);
//    weight packing (reidmi_vit_weights_pack / reidmi_text_weights_pack).
REIDMI_API int reidmi_abi_version(void) { return 4; }
