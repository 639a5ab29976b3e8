// distlowp.hip — the reduced-precision distance mode of SURVEY.md §8b (reidmi_distmat ... mode):
// euclidean_distance (evaluate.py:7-13) with the q.g products on fp16 operands and fp32
// accumulation (the encoder's GEMM, v_mfma_f32_16x16x32_f16), the squared norms exact fp32:
//   out[i][j] = (||q_i||^2 + ||g_j||^2) - 2 fp16(q_i).fp16(g_j)
// Not bit-exact with the reference's fp32 distances (reidmi_distmat_f32 is): it is the mode a
// caller chooses for throughput, with the error bound the tests state.
#include "common.h"
#include "gemm.h"

extern "C" int reidmi_row_sqnorm_f32(const float* x, int64_t n, int64_t d, int64_t ldx, float* out, void* stream);

namespace reidmi {

__global__ __launch_bounds__(256) void rows_to_f16_kernel(const float* __restrict__ src, int64_t rows, int64_t cols,
                                                          int64_t lds, _Float16* __restrict__ dst, int64_t ldd) {
    // fp32 [rows][cols] -> fp16 [gridDim.x][ldd], one workgroup per destination row; padding
    // rows and columns are zero
    const int64_t r = blockIdx.x;
    const float* s = src + r * lds;
    _Float16* d = dst + r * ldd;
    for (int64_t c = threadIdx.x; c < ldd; c += 256) d[c] = (r < rows && c < cols) ? (_Float16)s[c] : (_Float16)0.0f;
}

struct LowpPlan {
    int64_t Dp, Gp, qh, gh, qq, gg, total;
};

static LowpPlan lowp_plan(int64_t Q, int64_t G, int64_t D) {
    LowpPlan p{};
    auto al = [](int64_t v) { return (v + 255) & ~(int64_t)255; };
    p.Dp = (D + 63) / 64 * 64;  // the GEMM's K step
    p.Gp = (G + 255) / 256 * 256;
    int64_t o = 0;
    p.qh = o; o = al(o + Q * p.Dp * 2);
    p.gh = o; o = al(o + p.Gp * p.Dp * 2);
    p.qq = o; o = al(o + Q * 4);
    p.gg = o; o = al(o + G * 4);
    p.total = o;
    return p;
}

}  // namespace reidmi

using namespace reidmi;

REIDMI_API int64_t reidmi_distmat_f16_workspace_bytes(int64_t Q, int64_t G, int64_t D) {
    if (Q < 0 || G < 0 || D <= 0) return -1;
    return lowp_plan(Q, G, D).total;
}

REIDMI_API int reidmi_distmat_f16(const float* q, int64_t Q, int64_t ldq, const float* g, int64_t G, int64_t ldg,
                                  int64_t D, float* out, int64_t ldo, void* ws, int64_t ws_bytes, void* stream) {
    RM_REQUIRE(Q >= 0 && G >= 0 && D > 0 && ldq >= D && ldg >= D && ldo >= G, "distmat_f16: bad shape");
    const LowpPlan p = lowp_plan(Q, G, D);
    RM_REQUIRE(ws != nullptr && ws_bytes >= p.total, "distmat_f16: workspace smaller than reidmi_distmat_f16_workspace_bytes");
    if (Q == 0 || G == 0) return OK;
    RM_REQUIRE(q && g && out, "distmat_f16: null operand");
    RM_REQUIRE(Q < (1ll << 31) && p.Gp < (1ll << 31), "distmat_f16: too many rows");
    hipStream_t s = (hipStream_t)stream;
    char* w = (char*)ws;
    _Float16* qh = (_Float16*)(w + p.qh);
    _Float16* gh = (_Float16*)(w + p.gh);
    float* qq = (float*)(w + p.qq);
    float* gg = (float*)(w + p.gg);
    hipLaunchKernelGGL(rows_to_f16_kernel, dim3((unsigned)Q), dim3(256), 0, s, q, Q, D, ldq, qh, p.Dp);
    RM_LAUNCHED();
    hipLaunchKernelGGL(rows_to_f16_kernel, dim3((unsigned)p.Gp), dim3(256), 0, s, g, G, D, ldg, gh, p.Dp);
    RM_LAUNCHED();
    int rc;
    // exact fp32 squared norms (backend.hip's fmaf chain over k)
    if ((rc = reidmi_row_sqnorm_f32(q, Q, D, ldq, qq, stream))) return rc;
    if ((rc = reidmi_row_sqnorm_f32(g, G, D, ldg, gg, stream))) return rc;
    // the products and the distance in one pass: the GEMM's epilogue writes
    // (||q_i||^2 + ||g_j||^2) - 2 q.g straight into out (no Q x G product buffer)
    EpiArgs ea{};
    ea.out = out;
    ea.ldc = ldo;
    ea.dist_rsq = qq;
    ea.dist_csq = gg;
    ea.dist_n = G;
    return gemm_f16(EPI_F32, qh, p.Dp, gh, p.Dp, Q, p.Gp, p.Dp, ea, s);
}
