// gemm.hip — bf16 MFMA GEMM (C = A . W^T) with fused epilogues; see gemm.h.
//
// Tiling (MI355X / gfx950): 128x128x64 block tile, 256 threads = 4 waves as 2x2, each
// wave owns 64x64 = 4x4 tiles of v_mfma_f32_16x16x32_bf16.  Operand tiles are staged
// global -> registers -> LDS (double-buffered, one barrier per K-step: the loads for
// tile k+1 are in flight while tile k is multiplied).  LDS rows are 128 B; 16-byte
// chunks are XOR-swizzled with (row>>1)&7 so the fragment reads (16 rows x 4 chunks per
// ds_read_b128 lane group) are bank-conflict free.  Operands are swapped in the MFMA
// (W fragment as A, activation fragment as B) so each lane ends up holding one output
// row and 4 consecutive output columns: epilogue loads/stores are 8-16 B per lane.
// Block ids are remapped XCD-contiguously (consecutive tiles of one A row panel share
// an XCD's L2).
#include "gemm.h"

#include <cstdlib>
#include <type_traits>
#include <mutex>
#include <vector>

namespace reidmi {

// ----------------------------------------------------------- live GEMM timing
// bench.py measures the roofline of the dominant kernel with HIP events recorded on the
// launch stream around each GEMM of the timed region (reidmi_prof_*).  Off by default.
namespace prof {
struct Rec {
    hipEvent_t a, b;
    double flops;
    int epi;
};
static bool enabled = false;
static std::mutex mu;
static std::vector<Rec> recs;
static std::vector<std::pair<hipEvent_t, hipEvent_t>> pool;
static size_t used = 0;
}  // namespace prof

// Tile selection: 0 = auto (>= 256 tiles of 256x256: v6; else v1), 1..6 force
// v1 (128x128), v2 (256x256), v3 (persistent), v4 (ping-pong), v5 (persistent ping-pong),
// v6 (v5 with deferred epilogue-store waits: +1-2 % on the K = 768 shapes); A/B-only:
// v7 (two 32-MFMA sections per K-step: 1-3 % SLOWER than v5/v6, kept as the measured
// negative), v8 / v9 (v6 with the residual epilogue loading 2 / 4 row groups per batch
// instead of all 8).  Set by reidmi_gemm_set_variant (tests / A-B timing in one process);
// the REIDMI_GEMM_VARIANT environment variable gives the initial value.
static int g_variant = -1;
static int variant() {
    if (g_variant < 0) {
        const char* e = getenv("REIDMI_GEMM_VARIANT");
        g_variant = e ? atoi(e) : 0;
    }
    return g_variant;
}

constexpr int GB_M = 128, GB_N = 128, GB_K = 64;

__device__ __forceinline__ int swz(int r, int kc) { return r * GB_K + ((kc ^ ((r >> 1) & 7)) << 3); }

// one v_cvt_pk_bf16_f32 (RNE, NaN-preserving) per pair
__device__ __forceinline__ uint32_t cvt_pk_bf16(float a, float b) {
    uint32_t r;
    asm("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

__device__ __forceinline__ uint2 pack_bf16x4(float a, float b, float c, float d) {
    return make_uint2(cvt_pk_bf16(a, b), cvt_pk_bf16(c, d));
}

__device__ __forceinline__ float quick_gelu(float x) {
    // x * sigmoid(1.702 x) = x / (1 + 2^(-1.702 log2(e) x))   (custom_clip_model.py:52-54)
    return x * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(x * -2.4554669595930157f));
}

// Two QuickGELUs with the multiplies and the add on packed-fp32 VALU (v_pk_mul_f32 /
// v_pk_add_f32); the same operations in the same order as quick_gelu, so bit-identical.
typedef float f32x2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2v quick_gelu2(f32x2v x) {
    const f32x2v y = x * -2.4554669595930157f;
    const f32x2v d = f32x2v{__builtin_amdgcn_exp2f(y.x), __builtin_amdgcn_exp2f(y.y)} + 1.0f;
    return x * f32x2v{__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
}

// One 16x16x32 MFMA on 16-byte fragments holding bf16 or (F16) fp16 values.
template <bool F16>
__device__ __forceinline__ f32x4 mfma16(const bf16x8& w, const bf16x8& a, const f32x4& c) {
    if constexpr (F16)
        return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, w), __builtin_bit_cast(f16x8, a), c, 0,
                                                      0, 0);
    else
        return __builtin_amdgcn_mfma_f32_16x16x32_bf16(w, a, c, 0, 0, 0);
}

// LayerNorm fold (see gemm.h EpiArgs) with the bias: acc <- rstd_m * acc + (-mean_m rstd_m
// * s_n + b'_n), two FMAs per element (bias b'_n of the lane's columns passed in bn).  Lane
// layout as epilogue_tile; rows past M read row M-1.
template <int NI>
__device__ __forceinline__ void ln_fold(f32x4 (&acc)[NI][4], const float2* __restrict__ rowstat,
                                        const float* __restrict__ colsum, const float4 (&bn)[4], int64_t mrow,
                                        int ncol, int64_t M) {
    const int lane = threadIdx.x & 63;
    const int cq = (lane >> 4) * 4;
    float4 sn[4];
#pragma unroll
    for (int j = 0; j < 4; j++) sn[j] = *(const float4*)(colsum + ncol + j * 16 + cq);
    float2 rs[NI];
#pragma unroll
    for (int i = 0; i < NI; i++) {
        int64_t m = mrow + i * 16 + (lane & 15);
        rs[i] = rowstat[m < M ? m : M - 1];
    }
#pragma unroll
    for (int i = 0; i < NI; i++)
#pragma unroll
        for (int j = 0; j < 4; j++) {
            acc[i][j][0] = __builtin_fmaf(rs[i].x, acc[i][j][0], __builtin_fmaf(rs[i].y, sn[j].x, bn[j].x));
            acc[i][j][1] = __builtin_fmaf(rs[i].x, acc[i][j][1], __builtin_fmaf(rs[i].y, sn[j].y, bn[j].y));
            acc[i][j][2] = __builtin_fmaf(rs[i].x, acc[i][j][2], __builtin_fmaf(rs[i].y, sn[j].z, bn[j].z));
            acc[i][j][3] = __builtin_fmaf(rs[i].x, acc[i][j][3], __builtin_fmaf(rs[i].y, sn[j].w, bn[j].w));
        }
}

// Epilogue of one wave's output block: NI row groups x 4 column groups of 16x16, lane
// holding C[m][nb..nb+3] with m = mrow + i*16 + (lane&15), nb = ncol + j*16 + (lane>>4)*4
// (see gemm.h for the modes).  All loads are hoisted ahead of the stores they feed: bias
// once per tile, residual / pos-embed rows in batches of NB row groups — otherwise the
// compiler (which cannot prove `out` does not alias `bias`/`pos`) serialises one memory
// round trip per fragment.
template <int EPI, int NI, bool BIAS_DONE = false, int RNB = 2>
__device__ __forceinline__ void epilogue_tile(const EpiArgs& ea, f32x4 (&acc)[NI][4], int64_t mrow, int ncol,
                                              int64_t M, int N) {
    const int lane = threadIdx.x & 63;
    const int cq = (lane >> 4) * 4;
    if (!BIAS_DONE && EPI != EPI_PATCH && ea.bias != nullptr) {
        float4 b[4];
#pragma unroll
        for (int j = 0; j < 4; j++) b[j] = *(const float4*)(ea.bias + ncol + j * 16 + cq);
#pragma unroll
        for (int i = 0; i < NI; i++)
#pragma unroll
            for (int j = 0; j < 4; j++) {
                acc[i][j][0] += b[j].x;
                acc[i][j][1] += b[j].y;
                acc[i][j][2] += b[j].z;
                acc[i][j][3] += b[j].w;
            }
    }
    if constexpr (EPI == EPI_RESID_F16) {
        // Pair the fp32 accumulators first (v_permlane16_swap, see the bf16 path below; swap
        // whole uint4 images — per-element f32x4 read-modify-write around the builtin was
        // mis-lowered by hipcc 7.2, duplicating element 0 into elements 1..3):
        // afterwards lane group q holds columns colp(jp) .. +7 of its row in acc[i][2jp]
        // (first 4) and acc[i][2jp+1] (next 4) -> 16-byte fp16 loads and stores.
        const int q = lane >> 4;
#pragma unroll
        for (int i = 0; i < NI; i++)
#pragma unroll
            for (int jp = 0; jp < 2; jp++) {
                const uint4 a = __builtin_bit_cast(uint4, acc[i][2 * jp]);
                const uint4 c = __builtin_bit_cast(uint4, acc[i][2 * jp + 1]);
                const auto s0 = __builtin_amdgcn_permlane16_swap(a.x, c.x, false, false);
                const auto s1 = __builtin_amdgcn_permlane16_swap(a.y, c.y, false, false);
                const auto s2 = __builtin_amdgcn_permlane16_swap(a.z, c.z, false, false);
                const auto s3 = __builtin_amdgcn_permlane16_swap(a.w, c.w, false, false);
                acc[i][2 * jp] = __builtin_bit_cast(f32x4, make_uint4(s0[0], s1[0], s2[0], s3[0]));
                acc[i][2 * jp + 1] = __builtin_bit_cast(f32x4, make_uint4(s0[1], s1[1], s2[1], s3[1]));
            }
        _Float16* xo = (_Float16*)ea.out;
        auto colp = [&](int jp) { return ncol + (2 * jp + (q & 1)) * 16 + (q >> 1) * 8; };
        // row groups per batch (2*NB 16-byte loads in flight per lane).  The persistent tiles
        // load the whole residual block at once (RNB = 8: +6 % on out_proj at K = 768, where
        // the epilogue's HBM round trips are not amortised; v8 / v9 keep 2 / 4 for A/B).
        constexpr int NB = RNB < NI ? RNB : NI;
        auto store_batch = [&](int i0) {
#pragma unroll
            for (int ii = 0; ii < NB; ii++) {
                const int64_t m = mrow + (i0 + ii) * 16 + (lane & 15);
                const bool live = m < M;
                f16x8 h[2];
#pragma unroll
                for (int jp = 0; jp < 2; jp++) {
                    const f32x4 a = acc[i0 + ii][2 * jp], b = acc[i0 + ii][2 * jp + 1];
                    h[jp] = f16x8{(_Float16)a[0], (_Float16)a[1], (_Float16)a[2], (_Float16)a[3],
                                  (_Float16)b[0], (_Float16)b[1], (_Float16)b[2], (_Float16)b[3]};
                    if (live) *(f16x8*)(xo + m * ea.ldc + colp(jp)) = h[jp];
                }
                if (ea.pstat) {
                    // LayerNorm partials of the new fp16 row values over this wave's 64 columns
                    // (the 4 lane groups hold 16 each): sum, then the centred sum of squares
                    f32x2v sp = {0.f, 0.f};
#pragma unroll
                    for (int jp = 0; jp < 2; jp++)
#pragma unroll
                        for (int e = 0; e < 8; e += 2) sp += f32x2v{(float)h[jp][e], (float)h[jp][e + 1]};
                    float sum = sp.x + sp.y;
                    sum += __shfl_xor(sum, 16, 64);
                    sum += __shfl_xor(sum, 32, 64);
                    const f32x2v mu = {sum * (1.0f / 64), sum * (1.0f / 64)};
                    f32x2v dp = {0.f, 0.f};
#pragma unroll
                    for (int jp = 0; jp < 2; jp++)
#pragma unroll
                        for (int e = 0; e < 8; e += 2) {
                            const f32x2v d = f32x2v{(float)h[jp][e], (float)h[jp][e + 1]} - mu;
                            dp = __builtin_elementwise_fma(d, d, dp);
                        }
                    float m2 = dp.x + dp.y;
                    m2 += __shfl_xor(m2, 16, 64);
                    m2 += __shfl_xor(m2, 32, 64);
                    if (live && (lane >> 4) == 0) ea.pstat[(ncol >> 6) * ea.ldp + m] = make_float2(sum, m2);
                }
            }
        };
#pragma unroll
        for (int i0 = 0; i0 < NI; i0 += NB) {
            f16x8 xv[NB][2];
#pragma unroll
            for (int ii = 0; ii < NB; ii++) {
                int64_t m = mrow + (i0 + ii) * 16 + (lane & 15);
                m = m < M ? m : M - 1;  // clamped rows are loaded but not stored
#pragma unroll
                for (int jp = 0; jp < 2; jp++) xv[ii][jp] = *(const f16x8*)(xo + m * ea.ldc + colp(jp));
            }
            if (i0 > 0) store_batch(i0 - NB);
#pragma unroll
            for (int ii = 0; ii < NB; ii++)
#pragma unroll
                for (int jp = 0; jp < 2; jp++)
#pragma unroll
                    for (int e = 0; e < 4; e++) {
                        acc[i0 + ii][2 * jp][e] += (float)xv[ii][jp][e];
                        acc[i0 + ii][2 * jp + 1][e] += (float)xv[ii][jp][4 + e];
                    }
        }
        store_batch(NI - NB);
        return;
    }
    if constexpr (EPI == EPI_RESID_F32 || EPI == EPI_PATCH) {
        // software-pipelined: the loads of batch n+1 are issued before the stores of batch n,
        // so no wait ever covers a store (vmcnt retires in issue order).
        constexpr int NB = 2;  // row groups per batch: 8 float4 loads in flight per lane
        auto row_of = [&](int i) {
            const int64_t m = mrow + i * 16 + (lane & 15);
            return m < M ? m : M - 1;  // clamped rows are loaded but not stored
        };
        auto src_row = [&](int64_t m) -> const float* {
            if constexpr (EPI == EPI_RESID_F32) return (const float*)ea.out + m * ea.ldc + ncol + cq;
            else return ea.pos + (1 + (uint32_t)m % (uint32_t)ea.npatch) * (int64_t)N + ncol + cq;
        };
        auto store_batch = [&](int i0) {
#pragma unroll
            for (int ii = 0; ii < NB; ii++) {
                const int64_t m = mrow + (i0 + ii) * 16 + (lane & 15);
                if (m >= M) continue;
                if constexpr (EPI == EPI_RESID_F32) {
                    float* d = (float*)ea.out + m * ea.ldc + ncol + cq;
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        const f32x4 v = acc[i0 + ii][j];
                        *(float4*)(d + j * 16) = make_float4(v[0], v[1], v[2], v[3]);
                    }
                } else {  // patch rows of the fp16 residual stream
                    const uint32_t img = (uint32_t)m / (uint32_t)ea.npatch, p = (uint32_t)m - img * (uint32_t)ea.npatch;
                    _Float16* d = (_Float16*)ea.out + ((int64_t)img * ea.seq + 1 + p) * ea.ldc + ncol + cq;
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        const f32x4 v = acc[i0 + ii][j];
                        *(f16x4*)(d + j * 16) = f16x4{(_Float16)v[0], (_Float16)v[1], (_Float16)v[2], (_Float16)v[3]};
                    }
                }
            }
        };
#pragma unroll
        for (int i0 = 0; i0 < NI; i0 += NB) {
            float4 x[NB][4];
#pragma unroll
            for (int ii = 0; ii < NB; ii++) {
                const float* sp = src_row(row_of(i0 + ii));
#pragma unroll
                for (int j = 0; j < 4; j++) x[ii][j] = *(const float4*)(sp + j * 16);
            }
            if (i0 > 0) store_batch(i0 - NB);
#pragma unroll
            for (int ii = 0; ii < NB; ii++)
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    acc[i0 + ii][j][0] += x[ii][j].x;
                    acc[i0 + ii][j][1] += x[ii][j].y;
                    acc[i0 + ii][j][2] += x[ii][j].z;
                    acc[i0 + ii][j][3] += x[ii][j].w;
                }
        }
        store_batch(NI - NB);
        return;
    }
    if constexpr (EPI == EPI_F32) {
#pragma unroll
        for (int i = 0; i < NI; i++) {
            const int64_t m = mrow + i * 16 + (lane & 15);
            if (m >= M) continue;
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const f32x4 v = acc[i][j];
                *(float4*)((float*)ea.out + m * ea.ldc + ncol + j * 16 + cq) = make_float4(v[0], v[1], v[2], v[3]);
            }
        }
        return;
    }
    // bf16 outputs.  v^T tiles of the head split keep the scattered 2-byte stores.
    // Head split: the wave's 64 columns lie inside one of q / k / v (wd is a multiple of 64),
    // so the q/k/v selector and the column's offset inside it are wave-uniform; the token
    // index (b, t) of a row comes from one 32-bit division per row group (M < 2^31, checked
    // at launch) instead of 64-bit divisions per fragment.
    [[maybe_unused]] int qkv_sel = 0, qkv_c0 = 0;
    if constexpr (EPI == EPI_QKV) {
        const int wd = ea.heads * 64;
        const int nb = __builtin_amdgcn_readfirstlane(ncol + ea.n_off);
        qkv_sel = nb / wd;
        qkv_c0 = nb - qkv_sel * wd;
        if (qkv_sel == 2) {
            const uint32_t seq = (uint32_t)ea.seq;
            const int64_t lp = ea.lpad;
#pragma unroll
            for (int i = 0; i < NI; i++) {
                const int64_t m = mrow + i * 16 + (lane & 15);
                if (m >= M) continue;
                const uint32_t b = (uint32_t)m / seq, t = (uint32_t)m - b * seq;
                __bf16* vb = (__bf16*)ea.vt + (int64_t)b * ea.heads * 64 * lp + t;
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const f32x4 v = acc[i][j];
                    const int hd = qkv_c0 + j * 16 + cq;  // h * 64 + d
                    __bf16* dst = vb + (int64_t)hd * lp;
                    dst[0] = (__bf16)v[0];
                    dst[lp] = (__bf16)v[1];
                    dst[2 * lp] = (__bf16)v[2];
                    dst[3 * lp] = (__bf16)v[3];
                }
            }
            return;
        }
    }
    // Row-per-lane store widening (cdna_hip_programming.md T21, 16-lane form): lane group
    // q = lane>>4 holds columns 4q..4q+3 of fragments j and j+1; one v_permlane16_swap per
    // packed dword leaves groups 0/2 with 8 consecutive columns of fragment j and groups
    // 1/3 with 8 of fragment j+1 -> one 16-byte store per lane per fragment pair.
    const int q = lane >> 4;
#pragma unroll
    for (int i = 0; i < NI; i++) {
        const int64_t m = mrow + i * 16 + (lane & 15);
        [[maybe_unused]] __bf16* qkrow = nullptr;  // QKV: q / k row (b, h = 0, t)
        if constexpr (EPI == EPI_QKV) {
            const uint32_t seq = (uint32_t)ea.seq;
            const uint32_t b = (uint32_t)m / seq, t = (uint32_t)m - b * seq;
            qkrow = (__bf16*)(qkv_sel == 0 ? ea.q : ea.k) + ((int64_t)b * ea.heads * ea.seq + t) * 64;
        }
#pragma unroll
        for (int jp = 0; jp < 2; jp++) {
            f32x4 a = acc[i][2 * jp], c = acc[i][2 * jp + 1];
            if constexpr (EPI == EPI_GELU_BF16) {
#pragma unroll
                for (int e = 0; e < 4; e += 2) {
                    const f32x2v ga = quick_gelu2(f32x2v{a[e], a[e + 1]});
                    const f32x2v gc = quick_gelu2(f32x2v{c[e], c[e + 1]});
                    a[e] = ga.x;
                    a[e + 1] = ga.y;
                    c[e] = gc.x;
                    c[e + 1] = gc.y;
                }
            }
            const auto lo = __builtin_amdgcn_permlane16_swap(cvt_pk_bf16(a[0], a[1]), cvt_pk_bf16(c[0], c[1]), false, false);
            const auto hi = __builtin_amdgcn_permlane16_swap(cvt_pk_bf16(a[2], a[3]), cvt_pk_bf16(c[2], c[3]), false, false);
            const uint4 v = make_uint4(lo[0], hi[0], lo[1], hi[1]);
            const int col = ncol + (2 * jp + (q & 1)) * 16 + (q >> 1) * 8;
            if (m >= M) continue;
            if constexpr (EPI == EPI_QKV) {
                const int hd = qkv_c0 + (col - ncol);  // h * 64 + d
                *(uint4*)(qkrow + (int64_t)(hd >> 6) * ea.seq * 64 + (hd & 63)) = v;
            } else {
                *(uint4*)((__bf16*)ea.out + m * ea.ldc + col) = v;
            }
        }
    }
}

template <int EPI, bool F16>
__global__ __launch_bounds__(256, 2) void gemm_bf16_kernel(const __bf16* __restrict__ A, int64_t lda,
                                                           const __bf16* __restrict__ W, int64_t ldw, int64_t M,
                                                           int N, int K, EpiArgs ea, int tiles_n, int nwg) {
    __shared__ __attribute__((aligned(16))) __bf16 smem[2][2][GB_M * GB_K];
    const int bid = blockIdx.x;
    const int xcd = bid & 7, qq = nwg >> 3, rr = nwg & 7;
    const int wg = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (bid >> 3);
    const int tm = wg / tiles_n, tn = wg % tiles_n;
    const int64_t m0 = (int64_t)tm * GB_M;
    const int n0 = tn * GB_N;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid >> 1, wn = wid & 1;

    // per-thread staging slots: 4 x 16 B of A and of W per K-step
    const __bf16* gA[4];
    const __bf16* gW[4];
    int soff[4];
    bool aval[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
        const int c = tid + 256 * u, row = c >> 3, kc = c & 7;
        aval[u] = m0 + row < M;
        gA[u] = A + (aval[u] ? (m0 + row) : 0) * lda + kc * 8;
        gW[u] = W + (int64_t)(n0 + row) * ldw + kc * 8;
        soff[u] = swz(row, kc);
    }
    uint4 ra0, ra1, ra2, ra3, rw0, rw1, rw2, rw3;
#define GLOAD(k0)                                                                  \
    do {                                                                           \
        ra0 = aval[0] ? *(const uint4*)(gA[0] + (k0)) : make_uint4(0, 0, 0, 0);   \
        ra1 = aval[1] ? *(const uint4*)(gA[1] + (k0)) : make_uint4(0, 0, 0, 0);   \
        ra2 = aval[2] ? *(const uint4*)(gA[2] + (k0)) : make_uint4(0, 0, 0, 0);   \
        ra3 = aval[3] ? *(const uint4*)(gA[3] + (k0)) : make_uint4(0, 0, 0, 0);   \
        rw0 = *(const uint4*)(gW[0] + (k0));                                       \
        rw1 = *(const uint4*)(gW[1] + (k0));                                       \
        rw2 = *(const uint4*)(gW[2] + (k0));                                       \
        rw3 = *(const uint4*)(gW[3] + (k0));                                       \
    } while (0)
#define LSTORE(buf)                                                                \
    do {                                                                           \
        *(uint4*)(&smem[buf][0][soff[0]]) = ra0;                                   \
        *(uint4*)(&smem[buf][0][soff[1]]) = ra1;                                   \
        *(uint4*)(&smem[buf][0][soff[2]]) = ra2;                                   \
        *(uint4*)(&smem[buf][0][soff[3]]) = ra3;                                   \
        *(uint4*)(&smem[buf][1][soff[0]]) = rw0;                                   \
        *(uint4*)(&smem[buf][1][soff[1]]) = rw1;                                   \
        *(uint4*)(&smem[buf][1][soff[2]]) = rw2;                                   \
        *(uint4*)(&smem[buf][1][soff[3]]) = rw3;                                   \
    } while (0)

    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
        for (int j = 0; j < 4; j++) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    GLOAD(0);
    LSTORE(0);
    __syncthreads();
    const int nk = K / GB_K;
    for (int kt = 0; kt < nk; ++kt) {
        const int cur = kt & 1;
        if (kt + 1 < nk) GLOAD((kt + 1) * GB_K);
        const __bf16* sA = smem[cur][0];
        const __bf16* sW = smem[cur][1];
#pragma unroll
        for (int ks = 0; ks < 2; ks++) {
            bf16x8 af[4], wf[4];
            const int kc = ks * 4 + (lane >> 4);
#pragma unroll
            for (int i = 0; i < 4; i++) af[i] = *(const bf16x8*)(sA + swz(wm * 64 + i * 16 + (lane & 15), kc));
#pragma unroll
            for (int j = 0; j < 4; j++) wf[j] = *(const bf16x8*)(sW + swz(wn * 64 + j * 16 + (lane & 15), kc));
#pragma unroll
            for (int i = 0; i < 4; i++)
#pragma unroll
                for (int j = 0; j < 4; j++)
                    acc[i][j] = mfma16<F16>(wf[j], af[i], acc[i][j]);
        }
        if (kt + 1 < nk) LSTORE(cur ^ 1);
        __syncthreads();
    }

    // ------------------------------------------------------------------ epilogue
    if constexpr (F16) {
        if (ea.rowstat) {
            float4 bn[4];
            const int cq = (lane >> 4) * 4;
#pragma unroll
            for (int j = 0; j < 4; j++)
                bn[j] = ea.bias ? *(const float4*)(ea.bias + n0 + wn * 64 + j * 16 + cq) : make_float4(0.f, 0.f, 0.f, 0.f);
            ln_fold<4>(acc, ea.rowstat, ea.colsum, bn, m0 + wm * 64, n0 + wn * 64, M);
            epilogue_tile<EPI, 4, true>(ea, acc, m0 + wm * 64, n0 + wn * 64, M, N);
            return;
        }
    }
    epilogue_tile<EPI, 4>(ea, acc, m0 + wm * 64, n0 + wn * 64, M, N);
#undef GLOAD
#undef LSTORE
}


// ===================================================================== v2 tile
// 256x256x64 block tile, 512 threads = 8 waves as 2 (M) x 4 (N), 128x64 per wave
// (8x4 tiles of 16x16x32): half the LDS bytes per FLOP of the 64x64-per-wave v1 tile.
// Operands go HBM -> LDS by global_load_lds_dwordx4 (no VGPR staging): one wave-instruction
// fills 1 KiB = 8 LDS rows of 128 B, lane l -> row 8j + l/8, physical 16-B chunk l%8.  The
// (row>>1)&7 XOR swizzle is applied on the per-lane SOURCE address (logical chunk
// kc = physical ^ swz(row)), and the same XOR on the ds_read side, so LDS stays lane-linear
// and fragment reads stay conflict-free.  Two LDS stages (2 x 64 KiB): tile t+1 streams in
// while tile t is multiplied; one vmcnt(0) + barrier per K-step.  All LDS is one dynamic
// array (a second __shared__ object makes hipcc drain vmcnt before every ds_read).
constexpr int G2_M = 256, G2_N = 256;
constexpr int G2_STAGE = (G2_M + G2_N) * GB_K;  // bf16 elements per stage

typedef __attribute__((address_space(3))) void* lds_ptr_t;

template <int EPI>
__global__ __launch_bounds__(512, 2) void gemm2_bf16_kernel(const __bf16* __restrict__ A, int64_t lda,
                                                            const __bf16* __restrict__ W, int64_t ldw, int64_t M,
                                                            int N, int K, EpiArgs ea, int tiles_n, int nwg) {
    extern __shared__ __attribute__((aligned(16))) __bf16 lds2[];
    const int bid = blockIdx.x;
    const int xcd = bid & 7, qq = nwg >> 3, rr = nwg & 7;
    const int wg = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (bid >> 3);
    const int tm = wg / tiles_n, tn = wg % tiles_n;
    const int64_t m0 = (int64_t)tm * G2_M;
    const int n0 = tn * G2_N;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wid >> 2, wn = wid & 3;

    // glds sources: wave wid fills 1-KiB pieces j = 4*wid + u (u < 4) of A and of W
    const __bf16* srcA[4];
    const __bf16* srcW[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
        const int j = wid * 4 + u;
        const int r = 8 * j + (lane >> 3);
        const int kc = (lane & 7) ^ ((r >> 1) & 7);
        int64_t gm = m0 + r;
        gm = gm < M ? gm : M - 1;  // rows past M read a valid row; their outputs are dropped
        srcA[u] = A + gm * lda + kc * 8;
        srcW[u] = W + (int64_t)(n0 + r) * ldw + kc * 8;
    }
#define G2_ISSUE(stage, k0)                                                                              \
    do {                                                                                                 \
        __bf16* base_ = lds2 + (stage) * G2_STAGE;                                                       \
        _Pragma("unroll") for (int u = 0; u < 4; u++) {                                                  \
            const int j = wid * 4 + u;                                                                   \
            __builtin_amdgcn_global_load_lds(srcA[u] + (k0), (lds_ptr_t)(base_ + j * 512), 16, 0, 0);    \
            __builtin_amdgcn_global_load_lds(srcW[u] + (k0), (lds_ptr_t)(base_ + G2_M * GB_K + j * 512), \
                                             16, 0, 0);                                                  \
        }                                                                                                \
    } while (0)

    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; i++)
#pragma unroll
        for (int j = 0; j < 4; j++) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    G2_ISSUE(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const int nk = K / GB_K;
    for (int kt = 0; kt < nk; ++kt) {
        const int cur = kt & 1;
        if (kt + 1 < nk) G2_ISSUE(cur ^ 1, (kt + 1) * GB_K);
        const __bf16* sA = lds2 + cur * G2_STAGE;
        const __bf16* sW = sA + G2_M * GB_K;
#pragma unroll
        for (int ks = 0; ks < 2; ks++) {
            const int kc = ks * 4 + (lane >> 4);
            bf16x8 wf[4];
#pragma unroll
            for (int j = 0; j < 4; j++) wf[j] = *(const bf16x8*)(sW + swz(wn * 64 + j * 16 + (lane & 15), kc));
            bf16x8 af[8];
#pragma unroll
            for (int i = 0; i < 8; i++) af[i] = *(const bf16x8*)(sA + swz(wm * 128 + i * 16 + (lane & 15), kc));
            __builtin_amdgcn_s_setprio(1);
#pragma unroll
            for (int i = 0; i < 8; i++)
#pragma unroll
                for (int j = 0; j < 4; j++)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], af[i], acc[i][j], 0, 0, 0);
            __builtin_amdgcn_s_setprio(0);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
#undef G2_ISSUE
    epilogue_tile<EPI, 8>(ea, acc, m0 + wm * 128, n0 + wn * 64, M, N);
}


// ===================================================================== v3 tile
// v2's 256x256x64 tile and LDS-DMA staging, made persistent and software-pipelined:
//  * grid = min(#tiles, 256) workgroups (one per CU); each XCD group (bid % 8) walks a
//    contiguous range of tiles (consecutive tiles share the A row panel in that XCD's L2);
//  * during the last K-step of a tile the first K-step of the workgroup's next tile is
//    already streaming into the free LDS stage, so a tile's prologue latency is hidden;
//  * inside a K-step the fragments of k-step 1 are read while the MFMAs of k-step 0 run.
// Same MFMA sequence per output element as v1/v2 -> bit-identical results.
template <int EPI>
__global__ __launch_bounds__(512, 2) void gemm3_bf16_kernel(const __bf16* __restrict__ A, int64_t lda,
                                                            const __bf16* __restrict__ W, int64_t ldw, int64_t M,
                                                            int N, int K, EpiArgs ea, int tiles_n, int ntiles) {
    extern __shared__ __attribute__((aligned(16))) __bf16 lds3[];
    const int G = gridDim.x;
    const int bid = blockIdx.x;
    // XCD group x = bid % ng owns tiles [lo_x, hi_x); its members j = bid / ng stride by its size
    const int ng = G < 8 ? G : 8;
    const int x = bid % ng, gx = G / ng + ((G % ng) > x ? 1 : 0);
    const int j = bid / ng;
    const int lo = (int)((int64_t)ntiles * x / ng), hi = (int)((int64_t)ntiles * (x + 1) / ng);
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wid >> 2, wn = wid & 3;
    const int nk = K / GB_K;

    // glds piece jj = 4*wid + u covers LDS rows 8jj..8jj+7; lane -> row 8jj + lane/8
    const int lrow = lane >> 3, lchunk = lane & 7;
    auto issue = [&](int tile, int k0, int stage) {
        const int64_t m0 = (int64_t)(tile / tiles_n) * G2_M;
        const int n0 = (tile % tiles_n) * G2_N;
        __bf16* base = lds3 + stage * G2_STAGE;
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int jj = wid * 4 + u;
            const int r = 8 * jj + lrow;
            const int kc = (lchunk ^ ((r >> 1) & 7)) * 8;
            int64_t gm = m0 + r;
            gm = gm < M ? gm : M - 1;
            __builtin_amdgcn_global_load_lds(A + gm * lda + k0 + kc, (lds_ptr_t)(base + jj * 512), 16, 0, 0);
            __builtin_amdgcn_global_load_lds(W + (int64_t)(n0 + r) * ldw + k0 + kc,
                                             (lds_ptr_t)(base + G2_M * GB_K + jj * 512), 16, 0, 0);
        }
    };

    int tile = lo + j;
    if (tile >= hi) return;
    int stage = 0;
    issue(tile, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (; tile < hi; tile += gx) {
        const int next = tile + gx;
        f32x4 acc[8][4];
#pragma unroll
        for (int i = 0; i < 8; i++)
#pragma unroll
            for (int jn = 0; jn < 4; jn++) acc[i][jn] = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int kt = 0; kt < nk; ++kt) {
            if (kt + 1 < nk) issue(tile, (kt + 1) * GB_K, stage ^ 1);
            else if (next < hi) issue(next, 0, stage ^ 1);
            const __bf16* sA = lds3 + stage * G2_STAGE;
            const __bf16* sW = sA + G2_M * GB_K;
            const int kc0 = lane >> 4, kc1 = 4 + (lane >> 4);
            bf16x8 wf0[4], wf1[4], a0[8], a1[8];
#pragma unroll
            for (int jn = 0; jn < 4; jn++) wf0[jn] = *(const bf16x8*)(sW + swz(wn * 64 + jn * 16 + (lane & 15), kc0));
#pragma unroll
            for (int i = 0; i < 8; i++) a0[i] = *(const bf16x8*)(sA + swz(wm * 128 + i * 16 + (lane & 15), kc0));
#pragma unroll
            for (int jn = 0; jn < 4; jn++) wf1[jn] = *(const bf16x8*)(sW + swz(wn * 64 + jn * 16 + (lane & 15), kc1));
            __builtin_amdgcn_s_setprio(1);
#pragma unroll
            for (int i = 0; i < 8; i++) {
                // k-step 1 fragment of row block i streams in behind k-step 0's MFMAs
                a1[i] = *(const bf16x8*)(sA + swz(wm * 128 + i * 16 + (lane & 15), kc1));
#pragma unroll
                for (int jn = 0; jn < 4; jn++)
                    acc[i][jn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf0[jn], a0[i], acc[i][jn], 0, 0, 0);
            }
#pragma unroll
            for (int i = 0; i < 8; i++)
#pragma unroll
                for (int jn = 0; jn < 4; jn++)
                    acc[i][jn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf1[jn], a1[i], acc[i][jn], 0, 0, 0);
            __builtin_amdgcn_s_setprio(0);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            stage ^= 1;
        }
        const int64_t m0 = (int64_t)(tile / tiles_n) * G2_M;
        const int n0 = (tile % tiles_n) * G2_N;
        epilogue_tile<EPI, 8>(ea, acc, m0 + wm * 128, n0 + wn * 64, M, N);
    }
}


// ===================================================================== v4 tile
// 256x256x64, 8 waves, LDS-DMA staging as v2, with a ping-pong section schedule: every
// K-tile is 4 LOAD sections (ds_read fragments of one 64x32 output quadrant, issue a share
// of the next K-tile's LDS-DMA, lgkmcnt(0)) interleaved with 4 COMPUTE sections (16
// register-only MFMAs), one workgroup barrier after each section.  Waves 4-7 start one
// barrier late, so on each SIMD (waves w and w+4) one wave's LOAD runs beside the other's
// COMPUTE.  Quadrant order (0,0),(0,1),(1,1),(1,0) reuses A or B fragments between
// sections (12+4+8+4 reads per K-tile).  Hazards (slot = barrier interval, group B = one
// slot behind): next-tile DMA is issued in LOAD 0/1 of tile t into the buffer last read in
// LOAD 3 of tile t-1 (retired by lgkmcnt(0) before its barrier); every wave drains its DMA
// with vmcnt(0) at the end of LOAD 3, a barrier before any wave's LOAD 0 of tile t+1.
// Same MFMA sequence per output element as v1-v3 -> bit-identical results.
template <int EPI>
__global__ __launch_bounds__(512, 2) void gemm4_bf16_kernel(const __bf16* __restrict__ A, int64_t lda,
                                                            const __bf16* __restrict__ W, int64_t ldw, int64_t M,
                                                            int N, int K, EpiArgs ea, int tiles_n, int nwg) {
    extern __shared__ __attribute__((aligned(16))) __bf16 lds4[];
    const int bid = blockIdx.x;
    const int xcd = bid & 7, qq = nwg >> 3, rr = nwg & 7;
    const int wg = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (bid >> 3);
    const int tm = wg / tiles_n, tn = wg % tiles_n;
    const int64_t m0 = (int64_t)tm * G2_M;
    const int n0 = tn * G2_N;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = wid >> 2, wc = wid & 3;

    // Region DMA: each operand stage is 4 regions of 128 LDS rows (16 pieces of 8 rows):
    //   A0 = rows {0..63, 128..191} (quadrant qm=0 of both wave rows), A1 = the other 128;
    //   B0 = W rows {wc*64 + 0..31}, B1 = W rows {wc*64 + 32..63}.
    // Wave w moves pieces 2w, 2w+1 of a region.  Piece p of region (half h) covers rows
    // A: 128*(p>>3) + 64*h + 8*(p&7) + lane/8;  B: 64*(p>>2) + 32*h + 8*(p&3) + lane/8.
    const __bf16* srcA[2][2];
    const __bf16* srcW[2][2];
    int offA[2][2], offW[2][2];
#pragma unroll
    for (int h = 0; h < 2; h++)
#pragma unroll
        for (int u = 0; u < 2; u++) {
            const int pc = 2 * wid + u;
            const int ra = 128 * (pc >> 3) + 64 * h + 8 * (pc & 7);
            const int rb = 64 * (pc >> 2) + 32 * h + 8 * (pc & 3);
            const int r1 = ra + (lane >> 3), r2 = rb + (lane >> 3);
            int64_t gm = m0 + r1;
            gm = gm < M ? gm : M - 1;
            srcA[h][u] = A + gm * lda + ((lane & 7) ^ ((r1 >> 1) & 7)) * 8;
            srcW[h][u] = W + (int64_t)(n0 + r2) * ldw + ((lane & 7) ^ ((r2 >> 1) & 7)) * 8;
            offA[h][u] = ra * GB_K;
            offW[h][u] = G2_M * GB_K + rb * GB_K;
        }
#define G4_ISSUE_A(stage, h, k0)                                                                             \
    _Pragma("unroll") for (int u = 0; u < 2; u++) __builtin_amdgcn_global_load_lds(                          \
        srcA[h][u] + (k0), (lds_ptr_t)(lds4 + (stage) * G2_STAGE + offA[h][u]), 16, 0, 0)
#define G4_ISSUE_W(stage, h, k0)                                                                             \
    _Pragma("unroll") for (int u = 0; u < 2; u++) __builtin_amdgcn_global_load_lds(                          \
        srcW[h][u] + (k0), (lds_ptr_t)(lds4 + (stage) * G2_STAGE + offW[h][u]), 16, 0, 0)
#define G4_BARRIER()                              \
    do {                                          \
        __builtin_amdgcn_sched_barrier(0);        \
        __builtin_amdgcn_s_barrier();             \
        __builtin_amdgcn_sched_barrier(0);        \
    } while (0)
#define G4_LDS_DONE() asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory")

    bf16x8 fa[4][2], fb[2][2];
    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; i++)
#pragma unroll
        for (int j = 0; j < 4; j++) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    auto load_a = [&](const __bf16* sA, int qm) {
#pragma unroll
        for (int i = 0; i < 4; i++)
#pragma unroll
            for (int ks = 0; ks < 2; ks++)
                fa[i][ks] = *(const bf16x8*)(sA + swz(wr * 128 + qm * 64 + i * 16 + (lane & 15), ks * 4 + (lane >> 4)));
    };
    auto load_b = [&](const __bf16* sW, int qn) {
#pragma unroll
        for (int j = 0; j < 2; j++)
#pragma unroll
            for (int ks = 0; ks < 2; ks++)
                fb[j][ks] = *(const bf16x8*)(sW + swz(wc * 64 + qn * 32 + j * 16 + (lane & 15), ks * 4 + (lane >> 4)));
    };
    auto compute = [&](int qm, int qn) {
#pragma unroll
        for (int ks = 0; ks < 2; ks++)
#pragma unroll
            for (int i = 0; i < 4; i++)
#pragma unroll
                for (int j = 0; j < 2; j++)
                    acc[qm * 4 + i][qn * 2 + j] = mfma16<false>(fb[j][ks], fa[i][ks], acc[qm * 4 + i][qn * 2 + j]);
    };

    const int nk = K / GB_K;
    // prologue: tile 0 whole, tile 1 without B0 (B0 of tile t+1 goes out in LOAD 0 of tile t)
    G4_ISSUE_A(0, 0, 0);
    G4_ISSUE_A(0, 1, 0);
    G4_ISSUE_W(0, 0, 0);
    G4_ISSUE_W(0, 1, 0);
    if (nk > 1) {
        G4_ISSUE_A(1, 0, GB_K);
        G4_ISSUE_W(1, 1, GB_K);
        G4_ISSUE_A(1, 1, GB_K);
        asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    if (wr == 1) G4_BARRIER();
    // K-tile t reads stage t&1; region R of stage t&1 is refilled with tile t+2 right after
    // its last read (LOAD 0: A0, B0; LOAD 1: B1; LOAD 2: A1; LOAD 3: B0 again):
    //   LOAD 0 issues B0(t+1)  [stage t+1's B0 last read in LOAD 3 of tile t-1]
    //   LOAD 1 issues A0(t+2), LOAD 2 issues B1(t+2), LOAD 3 issues A1(t+2)
    // At the end of LOAD 3 everything of tile t+1 must have landed: only the 3 regions of
    // tile t+2 (6 pieces per wave) may still be in flight -> vmcnt(6).
    auto kstep = [&](int kt, auto n1_tag, auto n2_tag) {
        constexpr bool N1 = decltype(n1_tag)::value;  // tile kt+1 exists
        constexpr bool N2 = decltype(n2_tag)::value;  // tile kt+2 exists
        const int buf = kt & 1;
        const __bf16* sA = lds4 + buf * G2_STAGE;
        const __bf16* sW = sA + G2_M * GB_K;
        // LOAD 0 / COMPUTE (0,0)
        load_a(sA, 0);
        load_b(sW, 0);
        if constexpr (N1) { G4_ISSUE_W(buf ^ 1, 0, (kt + 1) * GB_K); }
        G4_LDS_DONE();
        G4_BARRIER();
        compute(0, 0);
        G4_BARRIER();
        // LOAD 1 / COMPUTE (0,1)
        load_b(sW, 1);
        if constexpr (N2) { G4_ISSUE_A(buf, 0, (kt + 2) * GB_K); }
        G4_LDS_DONE();
        G4_BARRIER();
        compute(0, 1);
        G4_BARRIER();
        // LOAD 2 / COMPUTE (1,1)
        load_a(sA, 1);
        if constexpr (N2) { G4_ISSUE_W(buf, 1, (kt + 2) * GB_K); }
        G4_LDS_DONE();
        G4_BARRIER();
        compute(1, 1);
        G4_BARRIER();
        // LOAD 3 / COMPUTE (1,0)
        load_b(sW, 0);
        if constexpr (N2) { G4_ISSUE_A(buf, 1, (kt + 2) * GB_K); }
        G4_LDS_DONE();
        if constexpr (N2) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        else if constexpr (N1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        G4_BARRIER();
        compute(1, 0);
        G4_BARRIER();
    };
    using T_ = std::integral_constant<bool, true>;
    using F_ = std::integral_constant<bool, false>;
    int kt = 0;
    for (; kt + 2 < nk; ++kt) kstep(kt, T_{}, T_{});
    if (kt + 1 < nk) { kstep(kt, T_{}, F_{}); ++kt; }
    kstep(kt, F_{}, F_{});
    if (wr == 0) G4_BARRIER();
#undef G4_ISSUE_A
#undef G4_ISSUE_W
#undef G4_BARRIER
#undef G4_LDS_DONE
    epilogue_tile<EPI, 8>(ea, acc, m0 + wr * 128, n0 + wc * 64, M, N);
}

// ===================================================================== v5 tile
// v4's region-DMA ping-pong schedule made persistent (grid = min(#tiles, 256), tile walk
// as v3).  The two DMA streams — "+1" (region B0 of the next K-step) and "+2" (A0, B1, A1
// of the K-step after) — run over the workgroup's concatenated (tile, K-step) sequence, so
// while a tile's epilogue runs, the next tile's first two K-steps are already landing.
// The epilogue needs no barrier: group A runs it in the slot where group B computes the
// tile's last quadrant.  Same MFMA sequence per output as v1-v4 -> bit-identical.
//
// DEFER (variant 6): the epilogue's stores are not waited for by the next tile's first
// K-step.  vmcnt retires in issue order, so v5's first `vmcnt(6)` after an epilogue waits
// for every store the epilogue issued (one HBM write round trip per tile, with the MFMAs
// idle).  Here the next tile's first "+1" DMA (B0 of its K-step 1) is issued BEFORE the
// epilogue, and that step's wait counts the epilogue's memory instructions as allowed to be
// outstanding: vmcnt(6 + S (+1 bias DMA)), S = EpiVm<EPI>::count (checked against the ISA:
// global_load/store_dwordx4 per wave and tile).  Only after a full tile (no masked rows,
// so exactly S instructions were issued) and not for scattered-v^T QKV tiles; otherwise the
// plain vmcnt(6).  The bias is read from LDS by inline ds_read (the compiler would insert a
// vmcnt(0) before a ds_read of an LDS-DMA'd slot, draining the in-flight DMA every tile).
template <int EPI>
struct EpiVm {  // vector-memory instructions of one full-tile epilogue_tile<EPI, 8> per wave
    static constexpr int count = EPI == EPI_BF16 || EPI == EPI_GELU_BF16 || EPI == EPI_QKV ? 16
                                 : EPI == EPI_RESID_F16 || EPI == EPI_F32                 ? 32
                                                                                          : -1;
};

template <int EPI, bool DEFER, bool F16, int RNB = 8>
__global__ __launch_bounds__(512, 2) void gemm5_bf16_kernel(const __bf16* __restrict__ A, int64_t lda,
                                                            const __bf16* __restrict__ W, int64_t ldw, int64_t M,
                                                            int N, int K, EpiArgs ea, int tiles_n, int ntiles) {
    extern __shared__ __attribute__((aligned(16))) __bf16 lds5[];
    const int G = gridDim.x;
    const int bid = blockIdx.x;
    const int ng = G < 8 ? G : 8;
    const int xg = bid % ng, gx = G / ng + ((G % ng) > xg ? 1 : 0);
    const int lo = (int)((int64_t)ntiles * xg / ng), hi = (int)((int64_t)ntiles * (xg + 1) / ng);
    const int first = lo + bid / ng;
    if (first >= hi) return;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = wid >> 2, wc = wid & 3;
    const int nk = K / GB_K;

    // per-lane DMA geometry (see v4): piece pc = 2*wid + u of region half h
    int rowA[2][2], kcA[2][2], offA[2][2], offW[2][2];
    uint32_t offAb[2][2], offWb[2][2];  // byte offsets from the tile's (row 0, k0) element
#pragma unroll
    for (int h = 0; h < 2; h++)
#pragma unroll
        for (int u = 0; u < 2; u++) {
            const int pc = 2 * wid + u;
            const int ra = 128 * (pc >> 3) + 64 * h + 8 * (pc & 7);
            const int rb = 64 * (pc >> 2) + 32 * h + 8 * (pc & 3);
            const int r1 = ra + (lane >> 3), r2 = rb + (lane >> 3);
            rowA[h][u] = r1;
            kcA[h][u] = ((lane & 7) ^ ((r1 >> 1) & 7)) * 8;
            offAb[h][u] = (uint32_t)(r1 * (int)lda + kcA[h][u]) * 2u;
            offWb[h][u] = (uint32_t)(r2 * (int)ldw + ((lane & 7) ^ ((r2 >> 1) & 7)) * 8) * 2u;
            offA[h][u] = ra * GB_K;
            offW[h][u] = G2_M * GB_K + rb * GB_K;
        }
    // a DMA stream position: tile (m0, n0), K-step, and whether all 256 A rows exist
    struct Pos {
        int tile, kt;
        int64_t m0;
        int n0;
        bool full;
    };
    auto set_tile = [&](Pos& p, int tile) {
        p.tile = tile;
        p.kt = 0;
        p.m0 = (int64_t)(tile / tiles_n) * G2_M;
        p.n0 = (tile % tiles_n) * G2_N;
        p.full = p.m0 + G2_M <= M;
    };
    auto advance = [&](Pos& p) {
        if (++p.kt == nk) set_tile(p, p.tile + gx);
    };
    // uniform tile base + per-lane 32-bit element offset (SGPR base + VGPR offset form)
    auto issue_a = [&](int stage, int h, const Pos& p) {
        const __bf16* base = A + p.m0 * lda + p.kt * GB_K;
        if (p.full) {
#pragma unroll
            for (int u = 0; u < 2; u++)
                __builtin_amdgcn_global_load_lds((const char*)base + offAb[h][u],
                                                 (lds_ptr_t)(lds5 + stage * G2_STAGE + offA[h][u]), 16, 0, 0);
        } else {  // partial last row tile: rows >= M read row M-1 (never stored)
            const int lim = (int)(M - p.m0);
#pragma unroll
            for (int u = 0; u < 2; u++) {
                const int r = rowA[h][u] < lim ? rowA[h][u] : lim - 1;
                __builtin_amdgcn_global_load_lds((const char*)base + (uint32_t)(r * (int)lda + kcA[h][u]) * 2u,
                                                 (lds_ptr_t)(lds5 + stage * G2_STAGE + offA[h][u]), 16, 0, 0);
            }
        }
    };
    auto issue_w = [&](int stage, int h, const Pos& p) {
        const __bf16* base = W + (int64_t)p.n0 * ldw + p.kt * GB_K;
#pragma unroll
        for (int u = 0; u < 2; u++)
            __builtin_amdgcn_global_load_lds((const char*)base + offWb[h][u],
                                             (lds_ptr_t)(lds5 + stage * G2_STAGE + offW[h][u]), 16, 0, 0);
    };
#define G5_BARRIER()                              \
    do {                                          \
        __builtin_amdgcn_sched_barrier(0);        \
        __builtin_amdgcn_s_barrier();             \
        __builtin_amdgcn_sched_barrier(0);        \
    } while (0)
#define G5_LDS_DONE() asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory")

    bf16x8 fa[4][2], fb[2][2];
    f32x4 acc[8][4];
    auto load_a = [&](const __bf16* sA, int qm) {
#pragma unroll
        for (int i = 0; i < 4; i++)
#pragma unroll
            for (int ks = 0; ks < 2; ks++)
                fa[i][ks] = *(const bf16x8*)(sA + swz(wr * 128 + qm * 64 + i * 16 + (lane & 15), ks * 4 + (lane >> 4)));
    };
    auto load_b = [&](const __bf16* sW, int qn) {
#pragma unroll
        for (int j = 0; j < 2; j++)
#pragma unroll
            for (int ks = 0; ks < 2; ks++)
                fb[j][ks] = *(const bf16x8*)(sW + swz(wc * 64 + qn * 32 + j * 16 + (lane & 15), ks * 4 + (lane >> 4)));
    };
    auto compute = [&](int qm, int qn) {
#pragma unroll
        for (int ks = 0; ks < 2; ks++)
#pragma unroll
            for (int i = 0; i < 4; i++)
#pragma unroll
                for (int j = 0; j < 2; j++)
                    acc[qm * 4 + i][qn * 2 + j] = mfma16<F16>(fb[j][ks], fa[i][ks], acc[qm * 4 + i][qn * 2 + j]);
    };

    // Bias of the current tile: one LDS-DMA per wave at the tile's first K-step into the
    // wave's own 1 KB slot (lane l -> bias[n0 + 4l .. 4l+3]); issued before that step's
    // B0 DMA, so the step's vmcnt(6) retires it.  The epilogue reads it with ds_read.
    const bool has_bias = EPI != EPI_PATCH && ea.bias != nullptr;
    float* bias_slot = (float*)(lds5 + 2 * G2_STAGE) + wid * 256;
    // Folded LayerNorm (F16): colsum of the tile's 256 columns and (rstd, -mean rstd) of the
    // wave's 128 rows go to LDS by the same DMA at the tile's first K-step (the rowstat
    // buffer is padded to whole 256-row tiles, gemm.h).
    const bool fold = F16 && ea.rowstat != nullptr;
    float* cs_slot = bias_slot + 8 * 256;
    float* rs_slot = bias_slot + 16 * 256;
    // streams: p1 = step s+1 (region B0), p2 = step s+2 (A0, B1, A1); requires nk >= 2
    Pos p1, p2;
    {
        Pos p0;
        set_tile(p0, first);
        issue_a(0, 0, p0);
        issue_a(0, 1, p0);
        issue_w(0, 0, p0);
        issue_w(0, 1, p0);
        p1 = p0;
        advance(p1);  // step 1: always inside the first tile (nk >= 2)
        issue_a(1, 0, p1);
        issue_w(1, 1, p1);
        issue_a(1, 1, p1);
        p2 = p1;
        advance(p2);
        asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    }
    __syncthreads();
    if (wr == 1) G5_BARRIER();
    int buf = 0;
    constexpr bool CAN_DEFER = DEFER && EpiVm<EPI>::count > 0;
    bool deferred = false;  // the previous tile's epilogue stores may still be in flight
    for (int tile = first; tile < hi; tile += gx) {
#pragma unroll
        for (int i = 0; i < 8; i++)
#pragma unroll
            for (int j = 0; j < 4; j++) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int kt = 0; kt < nk; ++kt) {
            const bool has1 = p1.tile < hi, has2 = p2.tile < hi;
            const bool b0_early = CAN_DEFER && kt == 0 && tile != first;  // issued before the epilogue
            const __bf16* sA = lds5 + buf * G2_STAGE;
            const __bf16* sW = sA + G2_M * GB_K;
            // LOAD 0 / COMPUTE (0,0)
            load_a(sA, 0);
            load_b(sW, 0);
            if (kt == 0 && has_bias)
                __builtin_amdgcn_global_load_lds(ea.bias + (tile % tiles_n) * G2_N + lane * 4, (lds_ptr_t)bias_slot,
                                                 16, 0, 0);
            if constexpr (F16) {
                if (kt == 0 && fold) {
                    __builtin_amdgcn_global_load_lds(ea.colsum + (tile % tiles_n) * G2_N + lane * 4,
                                                     (lds_ptr_t)cs_slot, 16, 0, 0);
                    __builtin_amdgcn_global_load_lds((const float*)(ea.rowstat + (int64_t)(tile / tiles_n) * G2_M +
                                                                    wr * 128) + lane * 4,
                                                     (lds_ptr_t)rs_slot, 16, 0, 0);
                }
            }
            if (has1 && !b0_early) issue_w(buf ^ 1, 0, p1);
            G5_LDS_DONE();
            G5_BARRIER();
            compute(0, 0);
            G5_BARRIER();
            // LOAD 1 / COMPUTE (0,1)
            load_b(sW, 1);
            if (has2) issue_a(buf, 0, p2);
            G5_LDS_DONE();
            G5_BARRIER();
            compute(0, 1);
            G5_BARRIER();
            // LOAD 2 / COMPUTE (1,1)
            load_a(sA, 1);
            if (has2) issue_w(buf, 1, p2);
            G5_LDS_DONE();
            G5_BARRIER();
            compute(1, 1);
            G5_BARRIER();
            // LOAD 3 / COMPUTE (1,0)
            load_b(sW, 0);
            if (has2) {
                issue_a(buf, 1, p2);
                G5_LDS_DONE();
                if constexpr (CAN_DEFER) {
                    constexpr int S = EpiVm<EPI>::count;
                    if (kt == 0 && deferred) {  // + the first K-step's bias / colsum / rowstat DMAs
                        if (fold)
                            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(S + 9) : "memory");
                        else if (has_bias)
                            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(S + 7) : "memory");
                        else
                            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(S + 6) : "memory");
                    } else {
                        asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
                    }
                } else {
                    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
                }
            } else {
                G5_LDS_DONE();
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            G5_BARRIER();
            compute(1, 0);
            G5_BARRIER();
            advance(p1);
            advance(p2);
            buf ^= 1;
        }
        const int64_t m0 = (int64_t)(tile / tiles_n) * G2_M;
        const int n0 = (tile % tiles_n) * G2_N;
        if constexpr (CAN_DEFER) {
            deferred = false;
            if (p1.tile < hi) {  // a next tile exists: issue its K-step 1 B0 (skipped in its LOAD 0)
                issue_w(buf ^ 1, 0, p1);
                deferred = m0 + G2_M <= M;
                if constexpr (EPI == EPI_QKV) deferred = deferred && (n0 + ea.n_off) / (ea.heads * 64) != 2;
            }
        }
        if (has_bias) {
            float4 b[4];
            if constexpr (DEFER) {
                // inline ds_read: no compiler-inserted vmcnt(0) for the LDS-DMA'd slot (retired
                // by the tile's first K-step wait)
                const float* bp = bias_slot + wc * 64 + (lane >> 4) * 4;
                const uint32_t ba = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) float*)bp;
                asm volatile("ds_read_b128 %0, %1" : "=v"(b[0]) : "v"(ba) : "memory");
                asm volatile("ds_read_b128 %0, %1 offset:64" : "=v"(b[1]) : "v"(ba) : "memory");
                asm volatile("ds_read_b128 %0, %1 offset:128" : "=v"(b[2]) : "v"(ba) : "memory");
                asm volatile("ds_read_b128 %0, %1 offset:192" : "=v"(b[3]) : "v"(ba) : "memory");
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            } else {
#pragma unroll
                for (int j = 0; j < 4; j++) b[j] = *(const float4*)(bias_slot + wc * 64 + j * 16 + (lane >> 4) * 4);
            }
            if constexpr (F16) {
                // acc <- rstd * acc + (-mean rstd * s_n + b'_n); without a fold (rstd, s) = (1, 0):
                // fma(1, acc, fma(0, 0, b)) == acc + b exactly.  One branch-free update (a
                // branch on acc would duplicate the 128 accumulators).
                float4 sn[4];
                float2 rs[8];
                if (fold) {
                    if constexpr (DEFER) {
                        const uint32_t ca = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) float*)(
                            cs_slot + wc * 64 + (lane >> 4) * 4);
                        const uint32_t ra = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) float*)(
                            rs_slot + (lane & 15) * 2);
                        asm volatile("ds_read_b128 %0, %1" : "=v"(sn[0]) : "v"(ca) : "memory");
                        asm volatile("ds_read_b128 %0, %1 offset:64" : "=v"(sn[1]) : "v"(ca) : "memory");
                        asm volatile("ds_read_b128 %0, %1 offset:128" : "=v"(sn[2]) : "v"(ca) : "memory");
                        asm volatile("ds_read_b128 %0, %1 offset:192" : "=v"(sn[3]) : "v"(ca) : "memory");
                        asm volatile("ds_read_b64 %0, %1" : "=v"(rs[0]) : "v"(ra) : "memory");
                        asm volatile("ds_read_b64 %0, %1 offset:128" : "=v"(rs[1]) : "v"(ra) : "memory");
                        asm volatile("ds_read_b64 %0, %1 offset:256" : "=v"(rs[2]) : "v"(ra) : "memory");
                        asm volatile("ds_read_b64 %0, %1 offset:384" : "=v"(rs[3]) : "v"(ra) : "memory");
                        asm volatile("ds_read_b64 %0, %1 offset:512" : "=v"(rs[4]) : "v"(ra) : "memory");
                        asm volatile("ds_read_b64 %0, %1 offset:640" : "=v"(rs[5]) : "v"(ra) : "memory");
                        asm volatile("ds_read_b64 %0, %1 offset:768" : "=v"(rs[6]) : "v"(ra) : "memory");
                        asm volatile("ds_read_b64 %0, %1 offset:896" : "=v"(rs[7]) : "v"(ra) : "memory");
                        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                    } else {
#pragma unroll
                        for (int j = 0; j < 4; j++) sn[j] = *(const float4*)(cs_slot + wc * 64 + j * 16 + (lane >> 4) * 4);
#pragma unroll
                        for (int i = 0; i < 8; i++) rs[i] = *(const float2*)(rs_slot + (i * 16 + (lane & 15)) * 2);
                    }
                } else {
#pragma unroll
                    for (int j = 0; j < 4; j++) sn[j] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
                    for (int i = 0; i < 8; i++) rs[i] = make_float2(1.f, 0.f);
                }
#pragma unroll
                for (int i = 0; i < 8; i++)
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        acc[i][j][0] = __builtin_fmaf(rs[i].x, acc[i][j][0], __builtin_fmaf(rs[i].y, sn[j].x, b[j].x));
                        acc[i][j][1] = __builtin_fmaf(rs[i].x, acc[i][j][1], __builtin_fmaf(rs[i].y, sn[j].y, b[j].y));
                        acc[i][j][2] = __builtin_fmaf(rs[i].x, acc[i][j][2], __builtin_fmaf(rs[i].y, sn[j].z, b[j].z));
                        acc[i][j][3] = __builtin_fmaf(rs[i].x, acc[i][j][3], __builtin_fmaf(rs[i].y, sn[j].w, b[j].w));
                    }
            } else {
#pragma unroll
                for (int i = 0; i < 8; i++)
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        acc[i][j][0] += b[j].x;
                        acc[i][j][1] += b[j].y;
                        acc[i][j][2] += b[j].z;
                        acc[i][j][3] += b[j].w;
                    }
            }
        }
        epilogue_tile<EPI, 8, true, RNB>(ea, acc, m0 + wr * 128, n0 + wc * 64, M, N);
    }
    if (wr == 0) G5_BARRIER();
#undef G5_BARRIER
#undef G5_LDS_DONE
}

// v7: v5's persistent 256x256x64 tile and LDS-DMA streams with TWO sections per K-step
// instead of four: LOAD X reads A quadrant 0 and both W quadrants (16 ds_read_b128), COMPUTE X
// runs the 32 MFMAs of output quadrants (0,0),(0,1); LOAD Y reads A quadrant 1, COMPUTE Y
// runs (1,0),(1,1).  Each compute section is 512 MFMA cycles (v5: 256), so the loading
// partner's LDS latency, DMA issue and lgkmcnt drain fit inside it, at half the barriers.
// Region refill: A0/W0/W1 of a stage are last read in LOAD X of step s (both halves, one
// barrier apart) -> refilled for step s+2 in LOAD Y of step s; A1 last read in LOAD Y of
// step s -> refilled for step s+2 in LOAD X of step s+1.  Every wait is vmcnt(8) (plus the
// tile's bias/colsum/rowstat pieces at its first K-step).  Per accumulator the MFMA chain
// (K ascending) is v5's, so results are bit-identical.
template <int EPI, bool F16>
__global__ __launch_bounds__(512, 2) void gemm7_bf16_kernel(const __bf16* __restrict__ A, int64_t lda,
                                                            const __bf16* __restrict__ W, int64_t ldw, int64_t M,
                                                            int N, int K, EpiArgs ea, int tiles_n, int ntiles) {
    extern __shared__ __attribute__((aligned(16))) __bf16 lds5[];
    const int G = gridDim.x;
    const int bid = blockIdx.x;
    const int ng = G < 8 ? G : 8;
    const int xg = bid % ng, gx = G / ng + ((G % ng) > xg ? 1 : 0);
    const int lo = (int)((int64_t)ntiles * xg / ng), hi = (int)((int64_t)ntiles * (xg + 1) / ng);
    const int first = lo + bid / ng;
    if (first >= hi) return;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = wid >> 2, wc = wid & 3;
    const int nk = K / GB_K;

    int rowA[2][2], kcA[2][2], offA[2][2], offW[2][2];
    uint32_t offAb[2][2], offWb[2][2];
#pragma unroll
    for (int h = 0; h < 2; h++)
#pragma unroll
        for (int u = 0; u < 2; u++) {
            const int pc = 2 * wid + u;
            const int ra = 128 * (pc >> 3) + 64 * h + 8 * (pc & 7);
            const int rb = 64 * (pc >> 2) + 32 * h + 8 * (pc & 3);
            const int r1 = ra + (lane >> 3), r2 = rb + (lane >> 3);
            rowA[h][u] = r1;
            kcA[h][u] = ((lane & 7) ^ ((r1 >> 1) & 7)) * 8;
            offAb[h][u] = (uint32_t)(r1 * (int)lda + kcA[h][u]) * 2u;
            offWb[h][u] = (uint32_t)(r2 * (int)ldw + ((lane & 7) ^ ((r2 >> 1) & 7)) * 8) * 2u;
            offA[h][u] = ra * GB_K;
            offW[h][u] = G2_M * GB_K + rb * GB_K;
        }
    struct Pos {
        int tile, kt;
        int64_t m0;
        int n0;
        bool full;
    };
    auto set_tile = [&](Pos& p, int tile) {
        p.tile = tile;
        p.kt = 0;
        p.m0 = (int64_t)(tile / tiles_n) * G2_M;
        p.n0 = (tile % tiles_n) * G2_N;
        p.full = p.m0 + G2_M <= M;
    };
    auto advance = [&](Pos& p) {
        if (++p.kt == nk) set_tile(p, p.tile + gx);
    };
    auto issue_a = [&](int stage, int h, const Pos& p) {
        const __bf16* base = A + p.m0 * lda + p.kt * GB_K;
        if (p.full) {
#pragma unroll
            for (int u = 0; u < 2; u++)
                __builtin_amdgcn_global_load_lds((const char*)base + offAb[h][u],
                                                 (lds_ptr_t)(lds5 + stage * G2_STAGE + offA[h][u]), 16, 0, 0);
        } else {
            const int lim = (int)(M - p.m0);
#pragma unroll
            for (int u = 0; u < 2; u++) {
                const int r = rowA[h][u] < lim ? rowA[h][u] : lim - 1;
                __builtin_amdgcn_global_load_lds((const char*)base + (uint32_t)(r * (int)lda + kcA[h][u]) * 2u,
                                                 (lds_ptr_t)(lds5 + stage * G2_STAGE + offA[h][u]), 16, 0, 0);
            }
        }
    };
    auto issue_w = [&](int stage, int h, const Pos& p) {
        const __bf16* base = W + (int64_t)p.n0 * ldw + p.kt * GB_K;
#pragma unroll
        for (int u = 0; u < 2; u++)
            __builtin_amdgcn_global_load_lds((const char*)base + offWb[h][u],
                                             (lds_ptr_t)(lds5 + stage * G2_STAGE + offW[h][u]), 16, 0, 0);
    };
#define G7_BARRIER()                              \
    do {                                          \
        __builtin_amdgcn_sched_barrier(0);        \
        __builtin_amdgcn_s_barrier();             \
        __builtin_amdgcn_sched_barrier(0);        \
    } while (0)
#define G7_LDS_DONE() asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory")
#define G7_VM(n) asm volatile("s_waitcnt vmcnt(" #n ")" ::: "memory")

    bf16x8 fa[4][2], fb[4][2];
    f32x4 acc[8][4];
    auto load_a = [&](const __bf16* sA, int qm) {
#pragma unroll
        for (int i = 0; i < 4; i++)
#pragma unroll
            for (int ks = 0; ks < 2; ks++)
                fa[i][ks] = *(const bf16x8*)(sA + swz(wr * 128 + qm * 64 + i * 16 + (lane & 15), ks * 4 + (lane >> 4)));
    };
    auto load_b = [&](const __bf16* sW) {
#pragma unroll
        for (int j = 0; j < 4; j++)
#pragma unroll
            for (int ks = 0; ks < 2; ks++)
                fb[j][ks] = *(const bf16x8*)(sW + swz(wc * 64 + (j >> 1) * 32 + (j & 1) * 16 + (lane & 15),
                                                      ks * 4 + (lane >> 4)));
    };
    auto compute = [&](int qm) {
#pragma unroll
        for (int ks = 0; ks < 2; ks++)
#pragma unroll
            for (int i = 0; i < 4; i++)
#pragma unroll
                for (int j = 0; j < 4; j++)
                    acc[qm * 4 + i][j] = mfma16<F16>(fb[j][ks], fa[i][ks], acc[qm * 4 + i][j]);
    };

    const bool has_bias = EPI != EPI_PATCH && ea.bias != nullptr;
    float* bias_slot = (float*)(lds5 + 2 * G2_STAGE) + wid * 256;
    const bool fold = F16 && ea.rowstat != nullptr;
    float* cs_slot = bias_slot + 8 * 256;
    float* rs_slot = bias_slot + 16 * 256;
    // streams: pX = step s+1 (A1, issued in LOAD X), pY = step s+2 (A0, W0, W1, LOAD Y)
    Pos pX, pY;
    {
        Pos p0;
        set_tile(p0, first);
        issue_a(0, 0, p0);
        issue_w(0, 0, p0);
        issue_w(0, 1, p0);
        issue_a(0, 1, p0);
        pX = p0;
        advance(pX);  // step 1: inside the first tile (nk >= 2)
        issue_a(1, 0, pX);
        issue_w(1, 0, pX);
        issue_w(1, 1, pX);
        pY = pX;
        advance(pY);
        G7_VM(8);  // step 0's A0/W0/W1 landed
    }
    __syncthreads();
    if (wr == 1) G7_BARRIER();
    int buf = 0;
    for (int tile = first; tile < hi; tile += gx) {
#pragma unroll
        for (int i = 0; i < 8; i++)
#pragma unroll
            for (int j = 0; j < 4; j++) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int kt = 0; kt < nk; ++kt) {
            const bool hasX = pX.tile < hi, hasY = pY.tile < hi;
            const __bf16* sA = lds5 + buf * G2_STAGE;
            const __bf16* sW = sA + G2_M * GB_K;
            // LOAD X / COMPUTE X
            load_a(sA, 0);
            load_b(sW);
            int nb = 0;  // tile-start pieces (bias, colsum, rowstat), issued before pX's
            if (kt == 0 && has_bias) {
                __builtin_amdgcn_global_load_lds(ea.bias + (tile % tiles_n) * G2_N + lane * 4, (lds_ptr_t)bias_slot,
                                                 16, 0, 0);
                nb = 1;
            }
            if constexpr (F16) {
                if (kt == 0 && fold) {
                    __builtin_amdgcn_global_load_lds(ea.colsum + (tile % tiles_n) * G2_N + lane * 4,
                                                     (lds_ptr_t)cs_slot, 16, 0, 0);
                    __builtin_amdgcn_global_load_lds((const float*)(ea.rowstat + (int64_t)(tile / tiles_n) * G2_M +
                                                                    wr * 128) + lane * 4,
                                                     (lds_ptr_t)rs_slot, 16, 0, 0);
                    nb += 2;
                }
            }
            nb = __builtin_amdgcn_readfirstlane(nb);
            if (hasX) issue_a(buf ^ 1, 1, pX);
            G7_LDS_DONE();
            // A1 of this step (issued one LOAD X ago) landed
            if (!hasX) G7_VM(0);
            else if (nb == 0) G7_VM(8);
            else if (nb == 1) G7_VM(9);
            else G7_VM(11);
            G7_BARRIER();
            compute(0);
            G7_BARRIER();
            // LOAD Y / COMPUTE Y
            load_a(sA, 1);
            if (hasY) {
                issue_a(buf, 0, pY);
                issue_w(buf, 0, pY);
                issue_w(buf, 1, pY);
            }
            G7_LDS_DONE();
            // A0/W0/W1 of step s+1 (issued one LOAD Y ago) landed
            if (hasY) {
                if (nb == 0) G7_VM(8);
                else if (nb == 1) G7_VM(9);
                else G7_VM(11);
            } else if (hasX) {
                if (nb == 0) G7_VM(2);
                else if (nb == 1) G7_VM(3);
                else G7_VM(5);
            } else {
                G7_VM(0);
            }
            G7_BARRIER();
            compute(1);
            G7_BARRIER();
            advance(pX);
            advance(pY);
            buf ^= 1;
        }
        const int64_t m0 = (int64_t)(tile / tiles_n) * G2_M;
        const int n0 = (tile % tiles_n) * G2_N;
        if (has_bias) {
            // the tile-start pieces were retired by K-step 1's LOAD X wait (nk >= 2)
            float4 b[4];
            const float* bp = bias_slot + wc * 64 + (lane >> 4) * 4;
            const uint32_t ba = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) float*)bp;
            asm volatile("ds_read_b128 %0, %1" : "=v"(b[0]) : "v"(ba) : "memory");
            asm volatile("ds_read_b128 %0, %1 offset:64" : "=v"(b[1]) : "v"(ba) : "memory");
            asm volatile("ds_read_b128 %0, %1 offset:128" : "=v"(b[2]) : "v"(ba) : "memory");
            asm volatile("ds_read_b128 %0, %1 offset:192" : "=v"(b[3]) : "v"(ba) : "memory");
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if constexpr (F16) {
                float4 sn[4];
                float2 rs[8];
                if (fold) {
                    const uint32_t ca = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) float*)(
                        cs_slot + wc * 64 + (lane >> 4) * 4);
                    const uint32_t ra = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) float*)(
                        rs_slot + (lane & 15) * 2);
                    asm volatile("ds_read_b128 %0, %1" : "=v"(sn[0]) : "v"(ca) : "memory");
                    asm volatile("ds_read_b128 %0, %1 offset:64" : "=v"(sn[1]) : "v"(ca) : "memory");
                    asm volatile("ds_read_b128 %0, %1 offset:128" : "=v"(sn[2]) : "v"(ca) : "memory");
                    asm volatile("ds_read_b128 %0, %1 offset:192" : "=v"(sn[3]) : "v"(ca) : "memory");
                    asm volatile("ds_read_b64 %0, %1" : "=v"(rs[0]) : "v"(ra) : "memory");
                    asm volatile("ds_read_b64 %0, %1 offset:128" : "=v"(rs[1]) : "v"(ra) : "memory");
                    asm volatile("ds_read_b64 %0, %1 offset:256" : "=v"(rs[2]) : "v"(ra) : "memory");
                    asm volatile("ds_read_b64 %0, %1 offset:384" : "=v"(rs[3]) : "v"(ra) : "memory");
                    asm volatile("ds_read_b64 %0, %1 offset:512" : "=v"(rs[4]) : "v"(ra) : "memory");
                    asm volatile("ds_read_b64 %0, %1 offset:640" : "=v"(rs[5]) : "v"(ra) : "memory");
                    asm volatile("ds_read_b64 %0, %1 offset:768" : "=v"(rs[6]) : "v"(ra) : "memory");
                    asm volatile("ds_read_b64 %0, %1 offset:896" : "=v"(rs[7]) : "v"(ra) : "memory");
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                } else {
#pragma unroll
                    for (int j = 0; j < 4; j++) sn[j] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
                    for (int i = 0; i < 8; i++) rs[i] = make_float2(1.f, 0.f);
                }
#pragma unroll
                for (int i = 0; i < 8; i++)
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        acc[i][j][0] = __builtin_fmaf(rs[i].x, acc[i][j][0], __builtin_fmaf(rs[i].y, sn[j].x, b[j].x));
                        acc[i][j][1] = __builtin_fmaf(rs[i].x, acc[i][j][1], __builtin_fmaf(rs[i].y, sn[j].y, b[j].y));
                        acc[i][j][2] = __builtin_fmaf(rs[i].x, acc[i][j][2], __builtin_fmaf(rs[i].y, sn[j].z, b[j].z));
                        acc[i][j][3] = __builtin_fmaf(rs[i].x, acc[i][j][3], __builtin_fmaf(rs[i].y, sn[j].w, b[j].w));
                    }
            } else {
#pragma unroll
                for (int i = 0; i < 8; i++)
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        acc[i][j][0] += b[j].x;
                        acc[i][j][1] += b[j].y;
                        acc[i][j][2] += b[j].z;
                        acc[i][j][3] += b[j].w;
                    }
            }
        }
        epilogue_tile<EPI, 8, true>(ea, acc, m0 + wr * 128, n0 + wc * 64, M, N);
    }
    if (wr == 0) G7_BARRIER();
#undef G7_BARRIER
#undef G7_LDS_DONE
#undef G7_VM
}

template <int EPI, bool F16>
static int launch(const void* A, int64_t lda, const void* W, int64_t ldw, int64_t M, int64_t N, int64_t K,
                  const EpiArgs& ea, hipStream_t s) {
    int var = variant();
    if (F16 && var >= 2 && var <= 4) var = 0;  // fp16 operands: v1 / v5 / v6 / v7 only
    const int64_t tiles256 = (int64_t)ceil_div(M, G2_M) * (N / G2_N);
    if (N % G2_N == 0 && K >= 2 * GB_K && lda * G2_M < (1ll << 31) && ldw * G2_N < (1ll << 31) &&
        (var >= 5 || (var == 0 && tiles256 >= 256))) {
        const int tiles_m = ceil_div(M, G2_M), tiles_n = (int)(N / G2_N);
        const int64_t ntiles = (int64_t)tiles_m * tiles_n;
        RM_REQUIRE(ntiles < (1ll << 31), "gemm: grid too large");
        const size_t lds = 2 * (size_t)G2_STAGE * 2 + (F16 ? 3 : 1) * 8 * 256 * sizeof(float);
        static bool attr5 = false;
        if (!attr5) {
            RM_CHECK_HIP(hipFuncSetAttribute((const void*)gemm5_bf16_kernel<EPI, false, F16>,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
            RM_CHECK_HIP(hipFuncSetAttribute((const void*)gemm5_bf16_kernel<EPI, true, F16>,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
            attr5 = true;
        }
        const int grid = (int)(ntiles < 256 ? ntiles : 256);
        if (var == 7) {
            static bool attr7 = false;
            if (!attr7) {
                RM_CHECK_HIP(hipFuncSetAttribute((const void*)gemm7_bf16_kernel<EPI, F16>,
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
                attr7 = true;
            }
            hipLaunchKernelGGL((gemm7_bf16_kernel<EPI, F16>), dim3((unsigned)grid), dim3(512), lds, s,
                               (const __bf16*)A, lda, (const __bf16*)W, ldw, M, (int)N, (int)K, ea, tiles_n, (int)ntiles);
        } else if (var == 8 || var == 9) {  // A/B: the residual epilogue's old load batches
            static bool attr89 = false;
            if (!attr89) {
                RM_CHECK_HIP(hipFuncSetAttribute((const void*)gemm5_bf16_kernel<EPI, true, F16, 2>,
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
                RM_CHECK_HIP(hipFuncSetAttribute((const void*)gemm5_bf16_kernel<EPI, true, F16, 4>,
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
                attr89 = true;
            }
            if (var == 8)
                hipLaunchKernelGGL((gemm5_bf16_kernel<EPI, true, F16, 2>), dim3((unsigned)grid), dim3(512), lds, s,
                                   (const __bf16*)A, lda, (const __bf16*)W, ldw, M, (int)N, (int)K, ea, tiles_n,
                                   (int)ntiles);
            else
                hipLaunchKernelGGL((gemm5_bf16_kernel<EPI, true, F16, 4>), dim3((unsigned)grid), dim3(512), lds, s,
                                   (const __bf16*)A, lda, (const __bf16*)W, ldw, M, (int)N, (int)K, ea, tiles_n,
                                   (int)ntiles);
        } else if (var == 6 || var == 0)
            hipLaunchKernelGGL((gemm5_bf16_kernel<EPI, true, F16>), dim3((unsigned)grid), dim3(512), lds, s,
                               (const __bf16*)A, lda, (const __bf16*)W, ldw, M, (int)N, (int)K, ea, tiles_n, (int)ntiles);
        else
            hipLaunchKernelGGL((gemm5_bf16_kernel<EPI, false, F16>), dim3((unsigned)grid), dim3(512), lds, s,
                               (const __bf16*)A, lda, (const __bf16*)W, ldw, M, (int)N, (int)K, ea, tiles_n, (int)ntiles);
        RM_LAUNCHED();
        return OK;
    }
    if (!F16 && N % G2_N == 0 && var == 4) {
        const int tiles_m = ceil_div(M, G2_M), tiles_n = (int)(N / G2_N);
        const int64_t nwg = (int64_t)tiles_m * tiles_n;
        RM_REQUIRE(nwg < (1ll << 31), "gemm: grid too large");
        const size_t lds = 2 * (size_t)G2_STAGE * 2;
        static bool attr4 = false;
        if (!attr4) {
            RM_CHECK_HIP(hipFuncSetAttribute((const void*)gemm4_bf16_kernel<EPI>,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
            attr4 = true;
        }
        hipLaunchKernelGGL(gemm4_bf16_kernel<EPI>, dim3((unsigned)nwg), dim3(512), lds, s, (const __bf16*)A, lda,
                           (const __bf16*)W, ldw, M, (int)N, (int)K, ea, tiles_n, (int)nwg);
        RM_LAUNCHED();
        return OK;
    }
    if (!F16 && N % G2_N == 0 && var == 3) {
        const int tiles_m = ceil_div(M, G2_M), tiles_n = (int)(N / G2_N);
        const int64_t ntiles = (int64_t)tiles_m * tiles_n;
        RM_REQUIRE(ntiles < (1ll << 31), "gemm: grid too large");
        const size_t lds = 2 * (size_t)G2_STAGE * 2;
        static bool attr3 = false;
        if (!attr3) {
            RM_CHECK_HIP(hipFuncSetAttribute((const void*)gemm3_bf16_kernel<EPI>,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
            attr3 = true;
        }
        const int grid = (int)(ntiles < 256 ? ntiles : 256);
        hipLaunchKernelGGL(gemm3_bf16_kernel<EPI>, dim3((unsigned)grid), dim3(512), lds, s, (const __bf16*)A, lda,
                           (const __bf16*)W, ldw, M, (int)N, (int)K, ea, tiles_n, (int)ntiles);
        RM_LAUNCHED();
        return OK;
    }
    if (!F16 && N % G2_N == 0 && var != 1 && (var == 2 || (int64_t)ceil_div(M, G2_M) * (N / G2_N) >= 512)) {
        const int tiles_m = ceil_div(M, G2_M), tiles_n = (int)(N / G2_N);
        const int64_t nwg = (int64_t)tiles_m * tiles_n;
        RM_REQUIRE(nwg < (1ll << 31), "gemm: grid too large");
        const size_t lds = 2 * (size_t)G2_STAGE * 2;
        static bool attr = false;
        if (!attr) {
            RM_CHECK_HIP(hipFuncSetAttribute((const void*)gemm2_bf16_kernel<EPI>,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
            attr = true;
        }
        hipLaunchKernelGGL(gemm2_bf16_kernel<EPI>, dim3((unsigned)nwg), dim3(512), lds, s, (const __bf16*)A, lda,
                           (const __bf16*)W, ldw, M, (int)N, (int)K, ea, tiles_n, (int)nwg);
        RM_LAUNCHED();
        return OK;
    }
    const int tiles_m = ceil_div(M, GB_M), tiles_n = (int)(N / GB_N);
    const int64_t nwg = (int64_t)tiles_m * tiles_n;
    RM_REQUIRE(nwg < (1ll << 31), "gemm: grid too large");
    hipLaunchKernelGGL((gemm_bf16_kernel<EPI, F16>), dim3((unsigned)nwg), dim3(256), 0, s, (const __bf16*)A, lda,
                       (const __bf16*)W, ldw, M, (int)N, (int)K, ea, tiles_n, (int)nwg);
    RM_LAUNCHED();
    return OK;
}

template <bool F16>
static int gemm_any(int epi, const void* A, int64_t lda, const void* W, int64_t ldw, int64_t M, int64_t N, int64_t K,
                    const EpiArgs& ea, hipStream_t s) {
    RM_REQUIRE(M >= 0 && N > 0 && K > 0, "gemm: bad shape");
    RM_REQUIRE((epi != EPI_QKV && epi != EPI_PATCH) || M < (1ll << 31), "gemm: head split / patch rows need M < 2^31");
    RM_REQUIRE(N % GB_N == 0 && K % GB_K == 0, "gemm: needs N % 128 == 0 and K % 64 == 0");
    RM_REQUIRE(lda % 8 == 0 && ldw % 8 == 0 && lda >= K && ldw >= K, "gemm: lda/ldw must be >= K and 16-byte rows");
    RM_REQUIRE((epi != EPI_BF16 && epi != EPI_GELU_BF16 && epi != EPI_RESID_F16) ||
                   (ea.ldc % 8 == 0 && ((uintptr_t)ea.out & 15) == 0),
               "gemm: bf16/fp16 output needs ldc % 8 == 0 and a 16-byte aligned base");
    if (M == 0) return OK;
    hipEvent_t ev_b = nullptr;
    if (prof::enabled) {
        std::lock_guard<std::mutex> g(prof::mu);
        if (prof::used == prof::pool.size()) {
            hipEvent_t a, b;
            RM_CHECK_HIP(hipEventCreate(&a));
            RM_CHECK_HIP(hipEventCreate(&b));
            prof::pool.push_back({a, b});
        }
        auto pr = prof::pool[prof::used++];
        prof::recs.push_back({pr.first, pr.second, 2.0 * (double)M * (double)N * (double)K, epi});
        RM_CHECK_HIP(hipEventRecord(pr.first, s));
        ev_b = pr.second;
    }
    int rc;
    if constexpr (F16) {
        switch (epi) {
            case EPI_BF16: rc = launch<EPI_BF16, true>(A, lda, W, ldw, M, N, K, ea, s); break;
            case EPI_GELU_BF16: rc = launch<EPI_GELU_BF16, true>(A, lda, W, ldw, M, N, K, ea, s); break;
            case EPI_QKV: rc = launch<EPI_QKV, true>(A, lda, W, ldw, M, N, K, ea, s); break;
            default: return fail(EINVAL_, "gemm_f16: epilogue must be EPI_BF16, EPI_GELU_BF16 or EPI_QKV");
        }
    } else {
        switch (epi) {
            case EPI_BF16: rc = launch<EPI_BF16, false>(A, lda, W, ldw, M, N, K, ea, s); break;
            case EPI_GELU_BF16: rc = launch<EPI_GELU_BF16, false>(A, lda, W, ldw, M, N, K, ea, s); break;
            case EPI_RESID_F32: rc = launch<EPI_RESID_F32, false>(A, lda, W, ldw, M, N, K, ea, s); break;
            case EPI_QKV: rc = launch<EPI_QKV, false>(A, lda, W, ldw, M, N, K, ea, s); break;
            case EPI_PATCH: rc = launch<EPI_PATCH, false>(A, lda, W, ldw, M, N, K, ea, s); break;
            case EPI_F32: rc = launch<EPI_F32, false>(A, lda, W, ldw, M, N, K, ea, s); break;
            case EPI_RESID_F16: rc = launch<EPI_RESID_F16, false>(A, lda, W, ldw, M, N, K, ea, s); break;
            default: return fail(EINVAL_, "gemm: unknown epilogue");
        }
    }
    if (ev_b) RM_CHECK_HIP(hipEventRecord(ev_b, s));
    return rc;
}

int gemm_bf16(int epi, const void* A, int64_t lda, const void* W, int64_t ldw, int64_t M, int64_t N, int64_t K,
              const EpiArgs& ea, hipStream_t s) {
    return gemm_any<false>(epi, A, lda, W, ldw, M, N, K, ea, s);
}

int gemm_f16(int epi, const void* A, int64_t lda, const void* W, int64_t ldw, int64_t M, int64_t N, int64_t K,
             const EpiArgs& ea, hipStream_t s) {
    RM_REQUIRE((ea.rowstat == nullptr) == (ea.colsum == nullptr), "gemm_f16: rowstat and colsum go together");
    RM_REQUIRE(ea.rowstat == nullptr || ea.bias != nullptr, "gemm_f16: a folded LayerNorm needs the folded bias");
    return gemm_any<true>(epi, A, lda, W, ldw, M, N, K, ea, s);
}

}  // namespace reidmi

using namespace reidmi;

REIDMI_API int reidmi_gemm_set_variant(int v) {
    RM_REQUIRE(v >= 0 && v <= 9, "gemm variant: 0 auto, 1 128x128, 2 256x256, 3 256x256 persistent, 4 ping-pong, "
                                 "5 persistent ping-pong, 6 = 5 with deferred epilogue-store waits, 7 = 5 with two sections per K-step, 8 / 9 = 6 with 2 / 4 (default 8) residual row groups per load batch");
    g_variant = v;
    return OK;
}

REIDMI_API int reidmi_prof_enable(int on) {
    std::lock_guard<std::mutex> g(prof::mu);
    prof::enabled = on != 0;
    prof::recs.clear();
    prof::used = 0;
    return OK;
}

// Sum of device time (ms), launch count and algorithmic FLOPs of the recorded GEMM launches
// with epilogue `epi` (-1: all).  Waits for the recorded events; then clears the record.
REIDMI_API int reidmi_prof_collect_min(int epi, double min_flops, double* total_ms, int64_t* count, double* flops) {
    std::lock_guard<std::mutex> g(prof::mu);
    double t = 0, f = 0;
    int64_t n = 0;
    for (auto& r : prof::recs) {
        if (epi >= 0 && r.epi != epi) continue;
        if (r.flops < min_flops) continue;
        RM_CHECK_HIP(hipEventSynchronize(r.b));
        float ms = 0;
        RM_CHECK_HIP(hipEventElapsedTime(&ms, r.a, r.b));
        t += ms;
        f += r.flops;
        n++;
    }
    if (total_ms) *total_ms = t;
    if (count) *count = n;
    if (flops) *flops = f;
    prof::recs.clear();
    prof::used = 0;
    return OK;
}

REIDMI_API int reidmi_prof_collect(int epi, double* total_ms, int64_t* count, double* flops) {
    return reidmi_prof_collect_min(epi, 0.0, total_ms, count, flops);
}

REIDMI_API int reidmi_gemm_f16(int epi, const void* A, int64_t lda, const void* W, int64_t ldw, int64_t M, int64_t N,
                               int64_t K, const float* bias, const void* rowstat, const float* colsum, void* out,
                               int64_t ldc, void* stream) {
    RM_REQUIRE(epi == EPI_BF16 || epi == EPI_GELU_BF16, "reidmi_gemm_f16: epi must be 0 (bf16) or 1 (gelu bf16)");
    EpiArgs ea{};
    ea.out = out;
    ea.ldc = ldc;
    ea.bias = bias;
    ea.rowstat = (const float2*)rowstat;
    ea.colsum = colsum;
    return gemm_f16(epi, A, lda, W, ldw, M, N, K, ea, (hipStream_t)stream);
}

REIDMI_API int reidmi_gemm_bf16(int epi, const void* A, int64_t lda, const void* W, int64_t ldw, int64_t M, int64_t N,
                                int64_t K, const float* bias, void* out, int64_t ldc, void* stream) {
    RM_REQUIRE(epi == EPI_BF16 || epi == EPI_GELU_BF16 || epi == EPI_RESID_F32 || epi == EPI_F32 || epi == EPI_RESID_F16,
               "reidmi_gemm_bf16: epi must be 0 (bf16), 1 (gelu bf16), 2 (residual f32), 5 (f32) or 6 (residual f16)");
    EpiArgs ea{};
    ea.out = out;
    ea.ldc = ldc;
    ea.bias = bias;
    return gemm_bf16(epi, A, lda, W, ldw, M, N, K, ea, (hipStream_t)stream);
}
