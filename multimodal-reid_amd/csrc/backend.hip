// backend.hip — retrieval back end of the CLIP-ReID eval path on gfx950.
//
//   reidmi_l2norm_f32      F.normalize(feats, p=2, dim=1)           evaluate.py:114
//   reidmi_distmat_f32     ||q||^2 + ||g||^2 - 2 q.g  (exact fp32)  evaluate.py:7-13, reranking.py:36-41
//   reidmi_topk_rows_f32   first k of np.argsort(row) (stable)      evaluate.py:40, reranking.py:48
//   reidmi_eval_rows       per-query CMC/AP of eval_func            evaluate.py:40-80
//
// Bit-exact contract with oracle/reid_oracle.c: every dot product / squared norm is an
// fmaf chain over k ascending.  The distance GEMM runs on v_mfma_f32_32x32x2_f32, whose
// result is bit-for-bit that chain (one rounding per product, k-pairs in order).
#include "common.h"

#include <algorithm>
#include <cmath>

namespace reidmi {

// --------------------------------------------------------------------------- norms
// R rows per R-thread workgroup, one row's fmaf chain per thread (k ascending, the distance
// kernel's arithmetic).  With 16-byte rows the row segments are staged through LDS 32 columns
// at a time by coalesced float4 loads (the next segment in flight while the current one is
// summed), instead of each thread walking its own row (uncoalesced).  R = 64: a Market gallery
// (15 913 rows) is 249 workgroups, not 63 on 256 CUs (rows_sqnorm_launch).
constexpr int RSQ_K = 32, RSQ_R = 64;
template <int R>
__global__ __launch_bounds__(R) void row_sqnorm_kernel(const float* __restrict__ x, int64_t n, int64_t d, int64_t ld,
                                                       float* __restrict__ out) {
    __shared__ float tile[R][RSQ_K + 1];
    const int64_t r0 = (int64_t)blockIdx.x * R, i = r0 + threadIdx.x;
    if ((ld & 3) != 0 || ((uintptr_t)x & 15) != 0 || d < RSQ_K) {  // uniform
        if (i >= n) return;
        const float* r = x + i * ld;
        float acc = 0.0f;
        for (int64_t k = 0; k < d; k++) acc = __builtin_fmaf(r[k], r[k], acc);
        out[i] = acc;
        return;
    }
    // float4 f = threadIdx.x + R u of a segment: row f / 8, columns 4 (f % 8) .. + 3
    constexpr int U = RSQ_K / 4;
    float4 v[U];
    auto load = [&](int64_t k0) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int f = threadIdx.x + R * u, row = f >> 3, c = (f & 7) * 4;
            const int64_t gi = r0 + row < n ? r0 + row : n - 1;
            v[u] = *(const float4*)(x + gi * ld + k0 + c);
        }
    };
    const int64_t nk = d / RSQ_K;
    float acc = 0.0f;
    load(0);
    for (int64_t kt = 0; kt < nk; kt++) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int f = threadIdx.x + R * u, row = f >> 3, c = (f & 7) * 4;
            tile[row][c] = v[u].x;
            tile[row][c + 1] = v[u].y;
            tile[row][c + 2] = v[u].z;
            tile[row][c + 3] = v[u].w;
        }
        __syncthreads();
        if (kt + 1 < nk) load((kt + 1) * RSQ_K);
#pragma unroll
        for (int k = 0; k < RSQ_K; k++) acc = __builtin_fmaf(tile[threadIdx.x][k], tile[threadIdx.x][k], acc);
        __syncthreads();
    }
    if (i >= n) return;
    const float* r = x + i * ld;
    for (int64_t k = nk * RSQ_K; k < d; k++) acc = __builtin_fmaf(r[k], r[k], acc);
    out[i] = acc;
}

static void rows_sqnorm_launch(const float* x, int64_t n, int64_t d, int64_t ld, float* out, hipStream_t s) {
    hipLaunchKernelGGL(row_sqnorm_kernel<RSQ_R>, dim3((unsigned)ceil_div(n, RSQ_R)), dim3(RSQ_R), 0, s, x, n, d, ld,
                       out);
}

// y = x / max(sqrt(ss), 1e-12): one workgroup per row, coalesced.
__global__ void row_scale_kernel(const float* __restrict__ x, const float* __restrict__ ss, int64_t d,
                                 int64_t ldx, float* __restrict__ y, int64_t ldy) {
    int64_t i = blockIdx.x;
    float nrm = __builtin_sqrtf(ss[i]);
    nrm = nrm < 1e-12f ? 1e-12f : nrm;
    for (int64_t k = threadIdx.x; k < d; k += blockDim.x) y[i * ldy + k] = x[i * ldx + k] / nrm;
}

// ------------------------------------------------------------------- distance GEMM
// 128x128 output tile per 256-thread workgroup (2x2 waves, 64x64 per wave as 2x2
// 32x32 MFMA tiles).  Operands staged k-major in LDS so each MFMA operand read is 32
// consecutive floats per half-wave.
constexpr int DM_BM = 128, DM_BN = 128, DM_BK = 16, DM_PAD = 4;

template <bool COSINE>
__global__ __launch_bounds__(256) void distmat_f32_kernel(
    const float* __restrict__ q, const float* __restrict__ g, const float* __restrict__ qq,
    const float* __restrict__ gg, int64_t Q, int64_t G, int64_t D, int64_t ldq, int64_t ldg,
    float* __restrict__ out, int64_t ldo) {
    __shared__ float sA[DM_BK][DM_BM + DM_PAD];
    __shared__ float sB[DM_BK][DM_BN + DM_PAD];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid >> 1, wn = wid & 1;
    const int64_t bm = (int64_t)blockIdx.y * DM_BM, bn = (int64_t)blockIdx.x * DM_BN;
    f32x16 acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
        for (int b = 0; b < 2; b++) acc[a][b] = f32x16{};
    for (int64_t k0 = 0; k0 < D; k0 += DM_BK) {
        // stage: 128 rows x 16 k per operand, 8 elements per thread, 16 threads per row
#pragma unroll
        for (int u = 0; u < 8; u++) {
            int e = tid + 256 * u;
            int r = e >> 4, kk = e & 15;
            int64_t gk = k0 + kk;
            int64_t qi = bm + r, gj = bn + r;
            sA[kk][r] = (qi < Q && gk < D) ? q[qi * ldq + gk] : 0.0f;
            sB[kk][r] = (gj < G && gk < D) ? g[gj * ldg + gk] : 0.0f;
        }
        __syncthreads();
#pragma unroll
        for (int s = 0; s < DM_BK / 2; s++) {
            const int kr = 2 * s + (lane >> 5);
            float a0 = sA[kr][wm * 64 + (lane & 31)];
            float a1 = sA[kr][wm * 64 + 32 + (lane & 31)];
            float b0 = sB[kr][wn * 64 + (lane & 31)];
            float b1 = sB[kr][wn * 64 + 32 + (lane & 31)];
            acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
            acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
            acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
            acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
        }
        __syncthreads();
    }
#pragma unroll
    for (int mt = 0; mt < 2; mt++)
#pragma unroll
        for (int nt = 0; nt < 2; nt++)
#pragma unroll
            for (int r = 0; r < 16; r++) {
                int64_t i = bm + wm * 64 + mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
                int64_t j = bn + wn * 64 + nt * 32 + (lane & 31);
                if (i < Q && j < G) {
                    if constexpr (COSINE) {
                        // evaluate.py:16-26: arccos(clip(q.g * (1/(|q||g|)), -1+1e-5, 1-1e-5))
                        const float c = acc[mt][nt][r] * (1.0f / (__builtin_sqrtf(qq[i]) * __builtin_sqrtf(gg[j])));
                        out[i * ldo + j] = acosf(fminf(fmaxf(c, -1.0f + 1e-5f), 1.0f - 1e-5f));
                    } else {
                        out[i * ldo + j] = __builtin_fmaf(-2.0f, acc[mt][nt][r], qq[i] + gg[j]);
                    }
                }
            }
}

// Pipelined variant (D, ldq, ldg multiples of 4, 16-byte aligned rows): K-step DM2_BK, two
// LDS stages, the next K-step's operands loaded as coalesced float4 into registers while the
// current one is multiplied, one barrier per K-step.
// LDS rows padded by 1 dword so the transposed scalar stores are conflict-free.  The MFMA
// sequence per output (k pairs ascending on v_mfma_f32_32x32x2_f32) is the one above, so the
// result is bit-identical to distmat_f32_kernel (and to the oracle's fmaf chain).
// K-step 16 (33 KB of LDS, 112 VGPRs): four workgroups per CU; K-step 32 ran two (66 KB) and
// was 5 % slower at MSMT17 / re-rank-chunk sizes (profiles/r02/distmat_kstep_ab.txt).  The
// macros are A/B hooks for tools/build_variant.py.
#ifndef DM2_BK_
#define DM2_BK_ 16
#endif
#ifndef DM2_MINWG_
#define DM2_MINWG_ 4
#endif
#ifndef DM2_BAND
#define DM2_BAND 4
#endif
#if !defined(REIDMI_TOOLS) && (DM2_BK_ != 16 || DM2_MINWG_ != 4 || DM2_BAND != 4 || defined(RS_STATS) || \
                               defined(RS_SINGLE_PASS) || defined(EV_STAMPS) || defined(EV_PREFETCH) || defined(EV_U1))
#error "backend.hip: DM2_* / RS_* / EV_* variants build only with -DREIDMI_TOOLS (never into libreidmi.so)"
#endif
constexpr int DM2_BK = DM2_BK_, DM2_LD = DM_BM + 1;
constexpr int DM2_F4 = DM2_BK / 4;            // float4 per operand row and K-step
constexpr int DM2_U = DM_BM * DM2_F4 / 256;   // float4 staging slots per thread and operand

template <bool COSINE, bool SYM = false>
__global__ __launch_bounds__(256, DM2_MINWG_) void distmat2_f32_kernel(
    const float* __restrict__ q, const float* __restrict__ g, const float* __restrict__ qq,
    const float* __restrict__ gg, int64_t Q, int64_t G, int64_t D, int64_t ldq, int64_t ldg,
    float* __restrict__ out, int64_t ldo) {
    __shared__ float sA[2][DM2_BK][DM2_LD];
    __shared__ float sB[2][DM2_BK][DM2_LD];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid >> 1, wn = wid & 1;
    // 1-D grid, XCD-contiguous: workgroups bid, bid+8, ... share an XCD (round-robin
    // dispatch) and get consecutive tiles, row tile fastest, so the row tiles of one gallery
    // panel run back to back on one XCD and its panel is fetched into that L2 once.
    const int64_t tiles_m = (Q + DM_BM - 1) / DM_BM;
    const int64_t nwg = (int64_t)gridDim.x;
    const int64_t bid = blockIdx.x, xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int64_t wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
    int64_t bm, bn;
    if constexpr (SYM) {
        // the self-distance of one row set (q == g): tiles (tm, tn) with tm <= tn only, column
        // panel tn holding tiles 0..tn (tn (tn + 1) / 2 tiles before it); the epilogue also
        // writes the mirrored tile.  Bit-for-bit symmetric: fma(a, b, c) == fma(b, a, c) in
        // every step of the chain, and qq[i] + gg[j] == qq[j] + gg[i] (same array).
        int64_t tn = (int64_t)((__builtin_sqrt(8.0 * (double)wg + 1.0) - 1.0) * 0.5);
        while ((tn + 1) * (tn + 2) / 2 <= wg) tn++;
        while (tn * (tn + 1) / 2 > wg) tn--;
        bm = (wg - tn * (tn + 1) / 2) * DM_BM;
        bn = tn * DM_BN;
    } else if (DM2_BAND > 0 && tiles_m > DM2_BAND) {
        // bands of DM2_BAND row tiles walked column-major: the tiles an XCD runs at once
        // form a DM2_BAND x (32 / DM2_BAND) block, so their output rows are few and long
        const int64_t per = (int64_t)DM2_BAND * ((G + DM_BN - 1) / DM_BN), band = wg / per, r = wg - band * per;
        const int64_t rows = tiles_m - band * DM2_BAND < DM2_BAND ? tiles_m - band * DM2_BAND : DM2_BAND;
        bm = (band * DM2_BAND + r % rows) * DM_BM;
        bn = (r / rows) * DM_BN;
    } else {
        bm = (wg % tiles_m) * DM_BM;
        bn = (wg / tiles_m) * DM_BN;
    }
    // staging slots: float4 f = tid + 256u -> row f / DM2_F4, k group (f % DM2_F4) * 4
    const float* pa[DM2_U];
    const float* pb[DM2_U];
    bool va[DM2_U], vb[DM2_U];
    int srow[DM2_U], sk[DM2_U];
#pragma unroll
    for (int u = 0; u < DM2_U; u++) {
        const int f = tid + 256 * u;
        srow[u] = f / DM2_F4;
        sk[u] = (f % DM2_F4) * 4;
        va[u] = bm + srow[u] < Q;
        vb[u] = bn + srow[u] < G;
        pa[u] = q + (va[u] ? bm + srow[u] : 0) * ldq + sk[u];
        pb[u] = g + (vb[u] ? bn + srow[u] : 0) * ldg + sk[u];
    }
    float4 ra[DM2_U], rb[DM2_U];
    auto gload = [&](int64_t k0) {
#pragma unroll
        for (int u = 0; u < DM2_U; u++) {
            const bool kin = k0 + sk[u] < D;  // D % 4 == 0: a float4 is wholly in or out
            ra[u] = va[u] && kin ? *(const float4*)(pa[u] + k0) : make_float4(0.f, 0.f, 0.f, 0.f);
            rb[u] = vb[u] && kin ? *(const float4*)(pb[u] + k0) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    };
    auto lstore = [&](int st) {
#pragma unroll
        for (int u = 0; u < DM2_U; u++) {
            sA[st][sk[u] + 0][srow[u]] = ra[u].x;
            sA[st][sk[u] + 1][srow[u]] = ra[u].y;
            sA[st][sk[u] + 2][srow[u]] = ra[u].z;
            sA[st][sk[u] + 3][srow[u]] = ra[u].w;
            sB[st][sk[u] + 0][srow[u]] = rb[u].x;
            sB[st][sk[u] + 1][srow[u]] = rb[u].y;
            sB[st][sk[u] + 2][srow[u]] = rb[u].z;
            sB[st][sk[u] + 3][srow[u]] = rb[u].w;
        }
    };
    f32x16 acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
        for (int b = 0; b < 2; b++) acc[a][b] = f32x16{};
    gload(0);
    lstore(0);
    __syncthreads();
    const int64_t nk = (D + DM2_BK - 1) / DM2_BK;
    for (int64_t kt = 0; kt < nk; kt++) {
        const int cur = (int)(kt & 1);
        if (kt + 1 < nk) gload((kt + 1) * DM2_BK);
#pragma unroll
        for (int s = 0; s < DM2_BK / 2; s++) {
            const int kr = 2 * s + (lane >> 5);
            const float a0 = sA[cur][kr][wm * 64 + (lane & 31)];
            const float a1 = sA[cur][kr][wm * 64 + 32 + (lane & 31)];
            const float b0 = sB[cur][kr][wn * 64 + (lane & 31)];
            const float b1 = sB[cur][kr][wn * 64 + 32 + (lane & 31)];
            acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
            acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
            acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
            acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
        }
        if (kt + 1 < nk) lstore(cur ^ 1);
        __syncthreads();
    }
#pragma unroll
    for (int mt = 0; mt < 2; mt++)
#pragma unroll
        for (int nt = 0; nt < 2; nt++)
#pragma unroll
            for (int r = 0; r < 16; r++) {
                int64_t i = bm + wm * 64 + mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
                int64_t j = bn + wn * 64 + nt * 32 + (lane & 31);
                if (i < Q && j < G) {
                    if constexpr (COSINE) {
                        const float c = acc[mt][nt][r] * (1.0f / (__builtin_sqrtf(qq[i]) * __builtin_sqrtf(gg[j])));
                        out[i * ldo + j] = acosf(fminf(fmaxf(c, -1.0f + 1e-5f), 1.0f - 1e-5f));
                    } else {
                        const float v = __builtin_fmaf(-2.0f, acc[mt][nt][r], qq[i] + gg[j]);
                        out[i * ldo + j] = v;
                        if (SYM && bm != bn) out[j * ldo + i] = v;  // the mirrored tile
                    }
                }
            }
}

static bool dm2_ok(const float* q, int64_t ldq, const float* g, int64_t ldg, int64_t D);

// Self-distance of x [N][D] (the one-call re-rank's N x N matrix, reranking.py:36-44): the
// upper-triangle tiles and their mirror images, half the FLOPs of distmat_launch(x, x), same
// bits.  ws: N floats.
int distmat_self_launch(const float* x, int64_t N, int64_t ldx, int64_t D, float* out, int64_t ldo, float* ws,
                        hipStream_t s) {
    RM_REQUIRE(N > 0 && D > 0 && ldx >= D && ldo >= N && ws != nullptr, "distmat_self: bad shape");
    rows_sqnorm_launch(x, N, D, ldx, ws, s);
    RM_LAUNCHED();
    if (!dm2_ok(x, ldx, x, ldx, D)) {
        dim3 grid(ceil_div(N, DM_BN), ceil_div(N, DM_BM));
        RM_REQUIRE(grid.y <= 65535, "distmat: too many query rows for one launch");
        hipLaunchKernelGGL(distmat_f32_kernel<false>, grid, dim3(256), 0, s, x, x, ws, ws, N, N, D, ldx, ldx, out, ldo);
    } else {
        const int64_t T = (N + DM_BM - 1) / DM_BM;
        const int64_t tiles = T * (T + 1) / 2;
        RM_REQUIRE(tiles < (1ll << 31), "distmat_self: too many tiles");
        hipLaunchKernelGGL((distmat2_f32_kernel<false, true>), dim3((unsigned)tiles), dim3(256), 0, s, x, x, ws, ws, N, N,
                           D, ldx, ldx, out, ldo);
    }
    RM_LAUNCHED();
    return OK;
}

static bool dm2_ok(const float* q, int64_t ldq, const float* g, int64_t ldg, int64_t D) {
    return D % 4 == 0 && ldq % 4 == 0 && ldg % 4 == 0 && ((uintptr_t)q & 15) == 0 && ((uintptr_t)g & 15) == 0;
}

// ---------------------------------------------------------------- key helpers
__device__ __forceinline__ bool key_less(float av, int ai, float bv, int bi) {
    return av < bv || (av == bv && ai < bi);
}

// In-LDS bitonic sort of (v,i) pairs, ascending by (v, i); P a power of two.
__device__ void bitonic_sort_kv(float* sv, int* si, int P) {
    for (int k = 2; k <= P; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int t = threadIdx.x; t < P; t += blockDim.x) {
                int o = t ^ j;
                if (o > t) {
                    bool up = (t & k) == 0;
                    float av = sv[t], bv = sv[o];
                    int ai = si[t], bi = si[o];
                    bool gt = key_less(bv, bi, av, ai);
                    if (gt == up) { sv[t] = bv; sv[o] = av; si[t] = bi; si[o] = ai; }
                }
            }
            __syncthreads();
        }
    }
}

__device__ __forceinline__ int pow2_ceil(int n) {
    int p = 1;
    while (p < n) p <<= 1;
    return p;
}

// --------------------------------------------------------------------- top-k
// Per row: k smallest (value, index) pairs in ascending order == np.argsort(kind="stable")[:k].
// Streams the row once; a candidate buffer in LDS collects elements under the running
// k-th key and is merged (bitonic) into the selection when it fills.  Optional per-row
// divisor implements reranking.py:46 (od[i,:] = D[i,:] / colmax[i] for symmetric D).
constexpr int TK_CAP = 2048, TK_CHUNK = 1024;

struct TkLds {
    float sv[TK_CAP];
    int si[TK_CAP];
    int s_cnt, s_nsel;
    float s_tv;
    int s_ti;
};

// The selection of one row by the whole workgroup: afterwards L.sv / L.si [0, min(K, cols))
// hold the K smallest (val(j), j) in ascending (value, index) order among the j with
// keep(v, j).  K <= TK_CAP - TK_CHUNK.
struct KeepAll {
    __device__ bool operator()(float, int) const { return true; }
};
template <typename VAL, typename KEEP = KeepAll>
__device__ void topk_row_dev(VAL val, int64_t cols, int K, TkLds& L, KEEP keep = KEEP{}) {
    if (threadIdx.x == 0) { L.s_cnt = 0; L.s_nsel = 0; L.s_tv = __builtin_inff(); L.s_ti = 0x7fffffff; }
    __syncthreads();
    for (int64_t c0 = 0; c0 < cols; c0 += TK_CHUNK) {
        const float tv = L.s_tv;
        const int ti = L.s_ti, nsel = L.s_nsel;
#pragma unroll
        for (int u = 0; u < TK_CHUNK / 256; u++) {
            int64_t j = c0 + u * 256 + threadIdx.x;
            if (j < cols) {
                const float v = val(j);
                if (key_less(v, (int)j, tv, ti) && keep(v, (int)j)) {
                    int p = atomicAdd(&L.s_cnt, 1);
                    L.sv[nsel + p] = v;
                    L.si[nsel + p] = (int)j;
                }
            }
        }
        __syncthreads();
        const bool last = c0 + TK_CHUNK >= cols;
        const int n = L.s_nsel + L.s_cnt;
        __syncthreads();  // every thread has read s_cnt before anyone appends again
        if (last || n > TK_CAP - TK_CHUNK) {
            const int P = pow2_ceil(n < 2 ? 2 : n);
            for (int t = n + threadIdx.x; t < P; t += blockDim.x) { L.sv[t] = __builtin_inff(); L.si[t] = 0x7fffffff; }
            __syncthreads();
            bitonic_sort_kv(L.sv, L.si, P);
            if (threadIdx.x == 0) {
                int ns = n < K ? n : K;
                L.s_nsel = ns;
                L.s_cnt = 0;
                if (ns == K) { L.s_tv = L.sv[K - 1]; L.s_ti = L.si[K - 1]; }
            }
            __syncthreads();
        }
    }
}

// K > TK_RUN (reranking.py:48's initial_rank for k1 or k2 beyond 1023): rounds of TK_RUN, each
// a fresh stream over the row keeping only the keys after the last one selected (keys are
// unique: the index breaks every tie), so the rounds concatenate to the stable argsort prefix.
constexpr int TK_RUN = TK_CAP - TK_CHUNK;

__global__ __launch_bounds__(256) void topk_rows_kernel(const float* __restrict__ x, int64_t cols, int64_t ld,
                                                        const float* __restrict__ row_div, int K,
                                                        int32_t* __restrict__ out_idx, float* __restrict__ out_val,
                                                        int64_t ldo) {
    __shared__ TkLds L;
    const int64_t row = blockIdx.x;
    const float* base = x + row * ld;
    const bool has_div = row_div != nullptr;
    const float dv = has_div ? row_div[row] : 1.0f;
    auto val = [&](int64_t j) {
        float v = base[j];
        if (has_div) v = v / dv;
        return v;
    };
    float lv = -__builtin_inff();
    int li = -1;
    for (int done = 0; done < K;) {
        const int kk = K - done < TK_RUN ? K - done : TK_RUN;
        if (done == 0)
            topk_row_dev(val, cols, kk, L);
        else
            topk_row_dev(val, cols, kk, L, [&](float v, int j) { return key_less(lv, li, v, j); });
        for (int r = threadIdx.x; r < kk; r += blockDim.x) {
            out_idx[row * ldo + done + r] = L.si[r];
            if (out_val) out_val[row * ldo + done + r] = L.sv[r];
        }
        lv = L.sv[kk - 1];
        li = L.si[kk - 1];
        done += kk;
        __syncthreads();  // every thread has read the selection before the next round refills it
    }
}

// ------------------------------------------------- re-rank R2 with an fp16 pre-filter
// The staged re-rank's initial_rank rows (reranking.py:45-48: od[i,:] = D[i,:] / max_j D[i,j]
// for the symmetric D, stable argsort, first K) without the exact N-wide distance row: the
// fp16 GEMM gives dot~_ij = x~_i . x~_j (x~ = fp16(x), fp32 accumulation) and
//   |d~_ij - d_ij| <= e_ij = 1.01 (c_rel n_i n_j + 2^-23 (s_i + s_j) + c_abs (n_i + n_j) + D 2^-49)
// with d~ = fma(-2, dot~, s_i + s_j), d the exact fp32 chain value (dist_exact, the distance
// kernel's bits), s = squared norms, n = sqrt(s), c_rel = 2 (2^-10 + 2^-22 + 2.02 D 2^-24) +
// 2.02 2^-23 (fp16 operand rounding 2^-11 relative + 2^-25 absolute per element, both
// accumulation chains, the final fma), c_abs = 2.01 2^-25 sqrt(D).  Then, with lo = d~ - e,
// hi = d~ + e:
//   * the K smallest (od, j) all satisfy d_j <= tau' = tau + |tau| 2^-21, tau = the K-th
//     smallest hi (K items have d <= hi <= tau; od = fl(d / r) is monotone and one rounding
//     cannot move a d above tau (1 + 2^-22) to an od at or below fl(tau / r)), and every such
//     item has lo <= d <= tau': the candidate set {j : lo_j <= tau'} contains them;
//   * the row max is attained among {j : hi_j >= max_k lo_k}.
// The candidates' exact distances then give the same rowmax and the same K indices as the
// full row, bit for bit.  Only hi reaches HBM (the GEMM's EPI_RRHI epilogue computes it from
// the product and the items' norms); the selection takes lo = hi - w_i with the row's width w_i
// >= hi_ij - lo_ij for every j (rr_width), which only widens both candidate sets.  A row whose
// candidate lists overflow, or with a non-finite bound or
// max, is marked in need[] for the exact rows (reranking.HipStages.rank_rows runs them through
// the exact distance kernel + selection).
constexpr int RS_CCAP = 2048, RS_MCAP = 512;
#ifndef DE_UNROLL
#define DE_UNROLL 16
#endif

__device__ __forceinline__ float dist_exact(const float* __restrict__ feat, int64_t ldf, int D,
                                            const float* __restrict__ sqn, int64_t i, int64_t c) {
    const float* a = feat + i * ldf;
    const float* b = feat + c * ldf;
    float acc = 0.0f;
    int k = 0;
    if ((ldf & 3) == 0) {
        // unrolled so that many row loads are in flight ahead of the (sequential) fma chain
#pragma unroll DE_UNROLL
        for (; k + 4 <= D; k += 4) {
            const float4 x = *(const float4*)(a + k), y = *(const float4*)(b + k);
            acc = __builtin_fmaf(x.x, y.x, acc);
            acc = __builtin_fmaf(x.y, y.y, acc);
            acc = __builtin_fmaf(x.z, y.z, acc);
            acc = __builtin_fmaf(x.w, y.w, acc);
        }
    }
    for (; k < D; k++) acc = __builtin_fmaf(a[k], b[k], acc);
    return __builtin_fmaf(-2.0f, acc, sqn[i] + sqn[c]);
}

__device__ __forceinline__ float block_max(float v, float* red) {
    v = wave_max(v);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    float m = red[0];
    for (int w = 1; w < (int)(blockDim.x >> 6); w++) m = fmaxf(m, red[w]);
    __syncthreads();
    return m;
}

// Width of the pair bound of row i: hi(i, j) - (exact distance lower bound) <= w_i for every j,
// from the largest norm and squared norm over the items (e is increasing in both; the margin
// covers the roundings of hi, of fl(dt - e) and of this subtraction, each <= 2^-24 of
// magnitudes <= 2.2 (s_i + s_max)).  For L2-normalised features (every n_j = 1) it is 2 e + a
// few ulps, the width of the per-pair bound.
__device__ __forceinline__ float rr_width(float s_i, float n_i, float n_max, float s_max, float c_rel, float c_abs,
                                          float c_d) {
    const float e = 1.01f * (__builtin_fmaf(c_rel * n_i, n_max, 0x1p-23f * (s_i + s_max)) + c_abs * (n_i + n_max) + c_d);
    return 2.0f * e * (1.0f + 0x1p-10f) + 0x1p-20f * (s_i + s_max + e);
}

// Rows of the k-reciprocal R2 from the pre-filter bounds hi ([rows][ldd] fp32, the EPI_RRHI
// GEMM epilogue: gemm.h rr_hi), lo = hi - w_i (rr_width): the K-th smallest hi bounds the K-th
// smallest exact distance, every item with lo <= that bound is a candidate of the top K, every
// item with hi >= the largest lo a candidate of the row max; both are recomputed exactly.
__global__ __launch_bounds__(256) void rank_select_kernel(const float* __restrict__ dot, int64_t ldd,
                                                          const float* __restrict__ feat, int64_t ldf, int D,
                                                          const float* __restrict__ sqn, const float* __restrict__ nrm,
                                                          int64_t row0, int64_t N, int K, float c_rel, float c_abs,
                                                          float c_d, const float* __restrict__ nmax2,
                                                          int32_t* __restrict__ rank_out,
                                                          float* __restrict__ rowmax_out, int32_t* __restrict__ need) {
    __shared__ TkLds L;
    __shared__ float cv[RS_CCAP];
    __shared__ int ci[RS_CCAP];
    __shared__ int mi[RS_MCAP];
    __shared__ int s_nc, s_nm, s_bad;
    __shared__ float red[4];
    const int64_t r = blockIdx.x, i = row0 + r;
    const float* drow = dot + r * ldd;
    const float w = rr_width(sqn[i], nrm[i], nmax2[0], nmax2[1], c_rel, c_abs, c_d);
    auto bounds = [&](int64_t j, float& lo, float& hi) {
        hi = drow[j];
        lo = hi - w;
    };
    if (threadIdx.x == 0) { s_nc = 0; s_nm = 0; s_bad = 0; }
    // pass A: tau = the K-th smallest upper bound; the largest lower bound
    topk_row_dev(
        [&](int64_t j) {
            float lo, hi;
            bounds(j, lo, hi);
            return hi;
        },
        N, K, L);
    const float tau = L.sv[K - 1];
    float ml = -__builtin_inff();
    bool bad = !(tau <= 3.0e38f && tau >= -3.0e38f);
    for (int64_t j = threadIdx.x; j < N; j += blockDim.x) {
        float lo, hi;
        bounds(j, lo, hi);
        ml = fmaxf(ml, lo);
        bad = bad || !(lo == lo && hi == hi && hi < __builtin_inff());
    }
    if (bad) s_bad = 1;
    const float mlo = block_max(ml, red);
    const float thr = tau + fabsf(tau) * 0x1p-21f + 1e-37f;
    // pass B: candidate lists
    if (!s_bad) {
        for (int64_t j = threadIdx.x; j < N; j += blockDim.x) {
            float lo, hi;
            bounds(j, lo, hi);
            if (lo <= thr) {
                const int p = atomicAdd(&s_nc, 1);
                if (p < RS_CCAP) ci[p] = (int)j;
            }
            if (hi >= mlo) {
                const int p = atomicAdd(&s_nm, 1);
                if (p < RS_MCAP) mi[p] = (int)j;
            }
        }
    }
    __syncthreads();
    const int nc = s_nc, nm = s_nm;
    bool exact = s_bad || nc > RS_CCAP || nm > RS_MCAP;
    float rmax = 0.0f;
    if (!exact) {
        float m = -__builtin_inff();
        for (int t = threadIdx.x; t < nm; t += blockDim.x) m = fmaxf(m, dist_exact(feat, ldf, D, sqn, i, mi[t]));
        rmax = block_max(m, red);
        exact = !(rmax > 0.0f && rmax < __builtin_inff());  // degenerate rows: the exact path
    }
    if (!exact) {
        for (int t = threadIdx.x; t < nc; t += blockDim.x) cv[t] = dist_exact(feat, ldf, D, sqn, i, ci[t]) / rmax;
        const int P = pow2_ceil(nc < 2 ? 2 : nc);
        for (int t = nc + threadIdx.x; t < P; t += blockDim.x) { cv[t] = __builtin_inff(); ci[t] = 0x7fffffff; }
        __syncthreads();
        bitonic_sort_kv(cv, ci, P);
        for (int t = threadIdx.x; t < K; t += blockDim.x) rank_out[r * K + t] = ci[t];
        if (threadIdx.x == 0) {
            rowmax_out[r] = rmax;
            need[r] = 0;
        }
        return;
    }
    // the row needs the exact path (its distances are too concentrated for the bound, or not
    // finite): the caller runs reidmi_rr_rank_rows' exact MFMA rows for the rows marked here
    if (threadIdx.x == 0) need[r] = 1;
}

// Keep the entries j of idx[0, n) with keep(j) (order preserved, in place); one full wave.
template <typename KEEP>
__device__ int compact_wave(int* idx, int n, KEEP keep) {
    const int lane = threadIdx.x & 63;
    int w = 0;
    for (int b = 0; b < n; b += 64) {
        const int t = b + lane;
        const int j = t < n ? idx[t] : 0;
        const bool k = t < n && keep(j);
        const uint64_t m = __ballot(k);
        if (k) idx[w + __popcll(m & ((1ull << lane) - 1))] = j;
        w += __popcll(m);
    }
    return w;
}

// Single-pass form of rank_select_kernel (same bound, same output bits): one stream over the
// row feeds the K-smallest-hi selection and both candidate lists at once, against the running
// thresholds -- the running K-th smallest hi only decreases and the running max lo only
// increases, so each list holds a superset of the final one; a list near capacity, and both
// lists at the end, are filtered against the current thresholds (exact set of the 3-pass form).
#ifndef RS1_CHUNK
#define RS1_CHUNK 1024
#endif
// chunk of the stream, selection buffer, candidate and max-list capacities
constexpr int RS1_CH = RS1_CHUNK, RS1_TKCAP = 2 * RS1_CH, RS1_CCAP = 2 * RS1_CH, RS1_MCAP = RS1_CH + RS1_CH / 2;
struct Rs1Lds {
    float sv[RS1_TKCAP];
    int si[RS1_TKCAP];
    int s_cnt, s_nsel;
    float s_tv;
    int s_ti;
};

__global__ __launch_bounds__(256) void rank_select1_kernel(const float* __restrict__ dot, int64_t ldd,
                                                           const float* __restrict__ feat, int64_t ldf, int D,
                                                           const float* __restrict__ sqn,
                                                           const float* __restrict__ nrm, int64_t row0, int64_t N,
                                                           int K, float c_rel, float c_abs, float c_d,
                                                           const float* __restrict__ nmax2,
                                                           int32_t* __restrict__ rank_out,
                                                           float* __restrict__ rowmax_out, int32_t* __restrict__ need) {
    __shared__ Rs1Lds L;
    __shared__ int ci[RS1_CCAP];
    __shared__ int mi[RS1_MCAP];
    __shared__ int s_nc, s_nm, s_bad;
    __shared__ float red[4];
    const int64_t r = blockIdx.x, i = row0 + r;
    const float* drow = dot + r * ldd;   // the bounds hi of the row (EPI_RRHI)
    const float w = rr_width(sqn[i], nrm[i], nmax2[0], nmax2[1], c_rel, c_abs, c_d);
    const int wv = threadIdx.x >> 6;
    auto bounds_v = [&](float hj, float& lo, float& hi) {
        hi = hj;
        lo = hj - w;
    };
    auto bounds = [&](int64_t j, float& lo, float& hi) { bounds_v(drow[j], lo, hi); };
    // chunk loads (see the stream below): thread t takes items c0 + 4 (t + 256 u) .. + 3, one
    // 16-byte load each (ldd % 4 == 0; a vector that starts below N ends below ldd)
    constexpr int U = RS1_CH / 1024;
    auto load = [&](int64_t c0, float4* d) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int64_t j = c0 + 4 * (u * 256 + threadIdx.x);
            d[u] = j < N ? *(const float4*)(drow + j) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    };
    auto thr_of = [](float tau) { return tau + fabsf(tau) * 0x1p-21f + 1e-37f; };
    // the max-list threshold starts at the first chunk's largest lo
    float ml = -__builtin_inff();
    for (int64_t j = threadIdx.x; j < N && j < RS1_CH; j += blockDim.x) {
        float lo, hi;
        bounds(j, lo, hi);
        ml = fmaxf(ml, lo);
    }
    float mlo = block_max(ml, red);
    if (threadIdx.x == 0) { L.s_cnt = 0; L.s_nsel = 0; L.s_tv = __builtin_inff(); L.s_ti = 0x7fffffff; s_nc = 0; s_nm = 0; s_bad = 0; }
    __syncthreads();
    bool bad = false, c_lost = false, m_lost = false;
    float thr = __builtin_inff();
    // the chunk loads run three chunks ahead of the selection (four register sets in turn)
    auto chunk = [&](int64_t c0, const float4* cd) {
        const float tv = L.s_tv;
        const int ti = L.s_ti, nsel = L.s_nsel;
#pragma unroll
        for (int v = 0; v < 4 * U; v++) {
            const int64_t j = c0 + 4 * ((v >> 2) * 256 + threadIdx.x) + (v & 3);
            if (j < N) {
                float lo, hi;
                const float4 q = cd[v >> 2];
                bounds_v((v & 3) == 0 ? q.x : (v & 3) == 1 ? q.y : (v & 3) == 2 ? q.z : q.w, lo, hi);
                ml = fmaxf(ml, lo);
                bad = bad || !(lo == lo && hi == hi && hi < __builtin_inff());
                if (key_less(hi, (int)j, tv, ti)) {
                    const int p = atomicAdd(&L.s_cnt, 1);
                    L.sv[nsel + p] = hi;
                    L.si[nsel + p] = (int)j;
                }
                if (!c_lost && lo <= thr) ci[atomicAdd(&s_nc, 1)] = (int)j;
                if (!m_lost && hi >= mlo) mi[atomicAdd(&s_nm, 1)] = (int)j;
            }
        }
        const float wm = wave_max(ml);
        if ((threadIdx.x & 63) == 0) red[wv] = wm;
        __syncthreads();
        const bool last = c0 + RS1_CH >= N;
        const int n = L.s_nsel + L.s_cnt, nc = s_nc, nm = s_nm;
        mlo = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
        __syncthreads();  // every thread has read the counters before anyone appends again
        // the selection is also merged before the candidate list is filtered, so that the
        // filter uses the current K-th bound (the selection buffer alone merges rarely)
        if (last || n > RS1_TKCAP - RS1_CH || (!c_lost && nc > RS1_CCAP - RS1_CH)) {
            const int P = pow2_ceil(n < 2 ? 2 : n);
            for (int t = n + threadIdx.x; t < P; t += blockDim.x) { L.sv[t] = __builtin_inff(); L.si[t] = 0x7fffffff; }
            __syncthreads();
            bitonic_sort_kv(L.sv, L.si, P);
            if (threadIdx.x == 0) {
                const int ns = n < K ? n : K;
                L.s_nsel = ns;
                L.s_cnt = 0;
                if (ns == K) { L.s_tv = L.sv[K - 1]; L.s_ti = L.si[K - 1]; }
            }
            __syncthreads();
        }
        if (L.s_nsel == K) thr = thr_of(L.s_tv);
        // filter the lists when the next chunk could overrun them, and at the end; a list
        // still too long afterwards is dropped and rebuilt by a second pass with the final
        // thresholds
        if (last || (!c_lost && nc > RS1_CCAP - RS1_CH) || (!m_lost && nm > RS1_MCAP - RS1_CH)) {
            if (wv == 0 && !c_lost) {
                const int k = compact_wave(ci, nc, [&](int j) {
                    float lo, hi;
                    bounds(j, lo, hi);
                    return lo <= thr;
                });
                if (threadIdx.x == 0) s_nc = k;
            } else if (wv == 1 && !m_lost) {
                const int k = compact_wave(mi, nm, [&](int j) {
                    float lo, hi;
                    bounds(j, lo, hi);
                    return hi >= mlo;
                });
                if (threadIdx.x == 64) s_nm = k;
            }
            __syncthreads();
            c_lost = c_lost || (!last && s_nc > RS1_CCAP - RS1_CH);
            m_lost = m_lost || (!last && s_nm > RS1_MCAP - RS1_CH);
            __syncthreads();  // every thread has read the counters before anyone appends again
        }
    };
    float4 xd[U], yd[U], zd[U], wd[U];
    load(0, xd);
    load(RS1_CH, yd);
    load(2 * RS1_CH, zd);
    for (int64_t c0 = 0; c0 < N; c0 += 4 * RS1_CH) {
        load(c0 + 3 * RS1_CH, wd);
        chunk(c0, xd);
        if (c0 + RS1_CH >= N) break;
        load(c0 + 4 * RS1_CH, xd);
        chunk(c0 + RS1_CH, yd);
        if (c0 + 2 * RS1_CH >= N) break;
        load(c0 + 5 * RS1_CH, yd);
        chunk(c0 + 2 * RS1_CH, zd);
        if (c0 + 3 * RS1_CH >= N) break;
        load(c0 + 6 * RS1_CH, zd);
        chunk(c0 + 3 * RS1_CH, wd);
    }
    if (bad) s_bad = 1;
    __syncthreads();
    if ((c_lost || m_lost) && !s_bad) {  // uniform
        if (threadIdx.x == 0) {
            if (c_lost) s_nc = 0;
            if (m_lost) s_nm = 0;
        }
        __syncthreads();
        for (int64_t j = threadIdx.x; j < N; j += blockDim.x) {
            float lo, hi;
            bounds(j, lo, hi);
            if (c_lost && lo <= thr) {
                const int p = atomicAdd(&s_nc, 1);
                if (p < RS1_CCAP) ci[p] = (int)j;
            }
            if (m_lost && hi >= mlo) {
                const int p = atomicAdd(&s_nm, 1);
                if (p < RS1_MCAP) mi[p] = (int)j;
            }
        }
        __syncthreads();
    }
    const float tau = L.sv[K - 1];
    const int nc = s_nc, nm = s_nm;
#ifdef RS_STATS
    if (threadIdx.x == 0 && (blockIdx.x % 1024) == 7)
        printf("RS row %lld nc %d nm %d clost %d mlost %d bad %d\n", (long long)i, nc, nm, (int)c_lost, (int)m_lost, s_bad);
#endif
    bool exact = s_bad || !(tau <= 3.0e38f && tau >= -3.0e38f) || nc > RS1_TKCAP || nm > RS1_MCAP;  // the sort runs in the selection buffer
    float rmax = 0.0f;
    if (!exact) {
        float m = -__builtin_inff();
        for (int t = threadIdx.x; t < nm; t += blockDim.x) m = fmaxf(m, dist_exact(feat, ldf, D, sqn, i, mi[t]));
        rmax = block_max(m, red);
        exact = !(rmax > 0.0f && rmax < __builtin_inff());  // degenerate rows: the exact path
    }
    if (!exact) {
        float* cv = L.sv;  // the selection buffer is free once tau is read
        for (int t = threadIdx.x; t < nc; t += blockDim.x) cv[t] = dist_exact(feat, ldf, D, sqn, i, ci[t]) / rmax;
        const int P = pow2_ceil(nc < 2 ? 2 : nc);
        for (int t = nc + threadIdx.x; t < P; t += blockDim.x) { cv[t] = __builtin_inff(); ci[t] = 0x7fffffff; }
        __syncthreads();
        bitonic_sort_kv(cv, ci, P);
        for (int t = threadIdx.x; t < K; t += blockDim.x) rank_out[r * K + t] = ci[t];
        if (threadIdx.x == 0) {
            rowmax_out[r] = rmax;
            need[r] = 0;
        }
        return;
    }
    if (threadIdx.x == 0) need[r] = 1;
}

// ------------------------------------------ R2 pre-filter with the selection in the GEMM
// The dense form above writes hi for every (row, item) pair and streams it back (N^2 fp32: 4 TB
// each way at N = 1M).  The sampled form keeps the selection's state out of HBM:
//  1. hi of each row against a sample of the items (every S-th item; EPI_RRHI, [rows][ns]);
//     rr_sample_kernel: U_r = the K-th smallest hi in the sample bounds tau_r (the K-th
//     smallest hi over all items) from above, and lb_r = max over the sample of lo = hi - w_r
//     bounds the row's largest lo from below;
//  2. the full GEMM with the EPI_RRSV epilogue appends to row r's list only the pairs with
//     hi <= hmax_r (every pair with lo <= thr(U_r)) or hi >= lb_r (gemm.h) -- a superset of both of rank_select1's final
//     candidate lists ({lo <= thr(tau)} and {hi >= max lo}), and it holds the K smallest hi
//     (hi <= tau <= U) and the largest hi (>= max lo >= lb): the list's K-th smallest hi is
//     tau itself and its largest hi the row's largest;
//  3. rank_select_sv_kernel: sorts the row's list by (hi, index), takes tau and max lo from it,
//     and runs rank_select1's exact tail (exact chain for both candidate lists, rowmax, stable
//     order by od = d / rowmax): the same rank_out / rowmax bits.
// A row whose list overflows RR_SV_CAP, holds a non-finite bound, or whose candidate lists
// exceed rank_select1's capacities is marked in need[] for the exact rows, as before.
constexpr int RR_SV_CAP = 4096;

__global__ __launch_bounds__(256) void rr_sample_kernel(const float* __restrict__ hs, int64_t lds, int64_t ns,
                                                        const float* __restrict__ sqn, const float* __restrict__ nrm,
                                                        const float* __restrict__ nmax2, int64_t row0, int K,
                                                        float c_rel, float c_abs, float c_d,
                                                        float4* __restrict__ meta, float* __restrict__ wrow,
                                                        int32_t* __restrict__ cnt, int cap) {
    __shared__ TkLds L;
    __shared__ float red[4];
    const int64_t r = blockIdx.x, i = row0 + r;
    const float* row = hs + r * lds;
    const float w = rr_width(sqn[i], nrm[i], nmax2[0], nmax2[1], c_rel, c_abs, c_d);
    float mx = -__builtin_inff();
    int bad = 0;
    for (int64_t j = threadIdx.x; j < ns; j += blockDim.x) {
        const float v = row[j];
        bad |= !(v < __builtin_inff());  // NaN or +inf
        mx = fmaxf(mx, v);
    }
    mx = block_max(mx, red);
    bad = __syncthreads_or(bad);
    topk_row_dev([&](int64_t j) { return row[j]; }, ns, K, L);
    if (threadIdx.x == 0) {
        const float U = L.sv[K - 1];
        const bool ok = !bad && ns >= K && U < 3.0e38f && U > -3.0e38f && mx < 3.0e38f;
        // the epilogue keeps a pair unless lb > hi > hmax: hmax bounds from above every hi whose
        // lo = fl(hi - w) is <= thr(U) (the widening covers the roundings of hi - w and of T + w)
        const float T = U + fabsf(U) * 0x1p-21f + 1e-37f;
        const float hmax = (T + w) + (fabsf(T) + w) * 0x1p-20f + 1e-37f;
        meta[r] = make_float4(sqn[i], nrm[i], hmax, mx - w);  // the survivor epilogue's row record
        wrow[r] = w;
        cnt[r] = ok ? 0 : cap + 1;
    }
}

__global__ __launch_bounds__(256) void rank_select_sv_kernel(const int32_t* __restrict__ cnt,
                                                             const int2* __restrict__ list, int cap,
                                                             const float* __restrict__ wrow,
                                                             const float* __restrict__ feat, int64_t ldf, int D,
                                                             const float* __restrict__ sqn, int64_t row0, int K,
                                                             int32_t* __restrict__ rank_out,
                                                             float* __restrict__ rowmax_out,
                                                             int32_t* __restrict__ need) {
    __shared__ float sv[RR_SV_CAP];
    __shared__ int si[RR_SV_CAP];
    __shared__ float red[4];
    __shared__ int s_nc, s_fm;
    const int64_t r = blockIdx.x, i = row0 + r;
    const int n = cnt[r];
    if (n > cap || n < K) {  // overflow, a non-finite bound, or (never for N >= K) too few
        if (threadIdx.x == 0) need[r] = 1;
        return;
    }
    const int2* lr = list + r * cap;
    const int P = pow2_ceil(n < 2 ? 2 : n);
    for (int t = threadIdx.x; t < P; t += blockDim.x) {
        if (t < n) {
            const int2 e = lr[t];
            sv[t] = __builtin_bit_cast(float, e.y);
            si[t] = e.x;
        } else {
            sv[t] = __builtin_inff();
            si[t] = 0x7fffffff;
        }
    }
    int bad = 0;
    for (int t = threadIdx.x; t < n; t += blockDim.x) bad |= !(sv[t] < __builtin_inff());  // NaN or +inf
    if (threadIdx.x == 0) { s_nc = 0; s_fm = n; }
    if (__syncthreads_or(bad)) {  // a non-finite bound: the exact path, as rank_select1
        if (threadIdx.x == 0) need[r] = 1;
        return;
    }
    bitonic_sort_kv(sv, si, P);  // ascending (hi, index)
    const float w = wrow[r];
    const float tau = sv[K - 1];
    const float th = tau + fabsf(tau) * 0x1p-21f + 1e-37f;  // rank_select1's thr_of
    const float mlo = sv[n - 1] - w;                         // the row's largest lo
    // candidate list = the prefix with lo = hi - w <= th; max list = the suffix with hi >= mlo
    int pc = 0, fm = n;
    for (int t = threadIdx.x; t < n; t += blockDim.x) {
        if (sv[t] - w <= th) pc = t + 1 > pc ? t + 1 : pc;
        if (sv[t] >= mlo) fm = t < fm ? t : fm;
    }
    atomicMax(&s_nc, pc);
    atomicMin(&s_fm, fm);
    __syncthreads();
    const int nc = s_nc, f0 = s_fm, nm = n - f0;
    bool exact = !(tau <= 3.0e38f && tau >= -3.0e38f) || nc > RS1_TKCAP || nm > RS1_MCAP;
    float rmax = 0.0f;
    if (!exact) {
        float m = -__builtin_inff();
        for (int t = f0 + threadIdx.x; t < n; t += blockDim.x) m = fmaxf(m, dist_exact(feat, ldf, D, sqn, i, si[t]));
        rmax = block_max(m, red);
        exact = !(rmax > 0.0f && rmax < __builtin_inff());  // degenerate rows: the exact path
    }
    if (!exact) {
        // the candidates are sv / si [0, nc): their exact od replaces the bound in place
        const int P2 = pow2_ceil(nc < 2 ? 2 : nc);
        __syncthreads();  // every thread is done reading sv / si [f0, n) above
        for (int t = threadIdx.x; t < P2; t += blockDim.x) {
            if (t < nc) {
                sv[t] = dist_exact(feat, ldf, D, sqn, i, si[t]) / rmax;
            } else {
                sv[t] = __builtin_inff();
                si[t] = 0x7fffffff;
            }
        }
        __syncthreads();
        bitonic_sort_kv(sv, si, P2);
        for (int t = threadIdx.x; t < K; t += blockDim.x) rank_out[r * K + t] = si[t];
        if (threadIdx.x == 0) {
            rowmax_out[r] = rmax;
            need[r] = 0;
        }
        return;
    }
    if (threadIdx.x == 0) need[r] = 1;
}

void rank_select_consts(int D, float c[3]);

int rr_sample_launch(const float* hs, int64_t lds, int64_t ns, const float* sqn, const float* nrm, const float* nmax2,
                     int64_t row0, int64_t rows, int K, int D, float4* meta, float* wrow, int32_t* cnt, int cap,
                     hipStream_t s) {
    RM_REQUIRE(K >= 1 && K <= 64 && ns >= K && rows >= 0 && nmax2, "rr_sample: bad arguments");
    if (rows == 0) return OK;
    float c[3];
    rank_select_consts(D, c);
    hipLaunchKernelGGL(rr_sample_kernel, dim3((unsigned)rows), dim3(256), 0, s, hs, lds, ns, sqn, nrm, nmax2, row0, K,
                       c[0], c[1], c[2], meta, wrow, cnt, cap);
    RM_LAUNCHED();
    return OK;
}

int rank_select_sv_launch(const int32_t* cnt, const int2* list, int cap, const float* wrow, const float* feat,
                          int64_t ldf, int D, const float* sqn, int64_t row0, int64_t rows, int K, int32_t* rank_out,
                          float* rowmax_out, int32_t* need, hipStream_t s) {
    RM_REQUIRE(K >= 1 && K <= 64 && cap >= 1 && cap <= RR_SV_CAP && rows >= 0, "rank_select_sv: bad arguments");
    if (rows == 0) return OK;
    hipLaunchKernelGGL(rank_select_sv_kernel, dim3((unsigned)rows), dim3(256), 0, s, cnt, list, cap, wrow, feat, ldf, D,
                       sqn, row0, K, rank_out, rowmax_out, need);
    RM_LAUNCHED();
    return OK;
}

// fp16 copy of the features for the pre-filter GEMM: [Np][Dp], zero-padded rows / columns;
// *range_ok cleared when an element is beyond +-2^15 (fp16 would overflow) or not finite.
__global__ void feat16_kernel(const float* __restrict__ x, int64_t N, int64_t D, int64_t ldx, _Float16* __restrict__ y,
                              int64_t Np, int64_t Dp, int32_t* __restrict__ range_ok) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= Np * Dp) return;
    const int64_t r = t / Dp, c = t - r * Dp;
    float v = 0.0f;
    if (r < N && c < D) {
        v = x[r * ldx + c];
        if (!(fabsf(v) <= 32768.0f)) { *range_ok = 0; v = 0.0f; }
    }
    y[t] = (_Float16)v;
}

// ------------------------------------------------------------------- eval rows
// numpy pairwise sum (PW_BLOCKSIZE 128, 8 accumulators) of an n-long float64 vector that
// is zero except at sorted positions pos(0..m) with values val(t): adding +0.0 is exact,
// so only the tree structure over the nonzeros matters.  Iterative post-order walk.
// POS / VAL: callables t -> int64 position / double value.
template <typename POS, typename VAL>
__device__ double leaf_sum(POS pos, VAL val, int lo, int hi, int64_t off, int64_t n) {
    if (n < 8) {
        double res = 0.0;
        for (int t = lo; t < hi; t++) res += val(t);
        return res;
    }
    // r[] indexed only by constants (a run-time index would put it in scratch memory, one
    // memory round trip per access): each accumulator adds v or +0.0, and r + 0.0 == r for
    // every r reachable here (all accumulators start at +0.0 and the values are positive)
    double r[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const int64_t main_end = n - (n % 8);
    int t = lo;
    for (; t < hi && pos(t) - off < main_end; t++) {
        const int p = (int)((pos(t) - off) & 7);
        const double v = val(t);
#pragma unroll
        for (int k = 0; k < 8; k++) r[k] += p == k ? v : 0.0;
    }
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; t < hi; t++) res += val(t);
    return res;
}

template <typename POS>
__device__ int lower_pos(POS pos, int lo, int hi, int64_t x) {
    while (lo < hi) {
        int mid = (lo + hi) >> 1;
        if (pos(mid) < x) lo = mid + 1; else hi = mid;
    }
    return lo;
}

// The walk's stack lives in LDS (`st`, PW_DEPTH frames, one walker lane): a private
// array indexed at run time would sit in scratch memory, one HBM round trip per access.
struct PwFrame {
    int64_t off, n, n2;
    int lo, hi, mid, stage;
    double left;
};
constexpr int PW_DEPTH = 48;

template <typename POS, typename VAL>
__device__ double pairwise_sparse(POS pos, VAL val, int m, int64_t n, PwFrame* st) {
    using Frame = PwFrame;
    int sp = 0;
    st[sp++] = Frame{0, n, 0, 0, m, 0, 0, 0.0};
    double ret = 0.0;
    while (sp > 0) {
        Frame& f = st[sp - 1];
        if (f.stage == 0) {
            if (f.lo == f.hi) { ret = 0.0; sp--; continue; }
            if (f.hi - f.lo == 1) { ret = val(f.lo); sp--; continue; }  // x + zeros == x in any order
            if (f.n <= 128) { ret = leaf_sum(pos, val, f.lo, f.hi, f.off, f.n); sp--; continue; }
            int64_t n2 = f.n / 2;
            n2 -= n2 % 8;
            f.n2 = n2;
            f.mid = lower_pos(pos, f.lo, f.hi, f.off + n2);
            f.stage = 1;
            Frame c{f.off, n2, 0, f.lo, f.mid, 0, 0, 0.0};
            st[sp++] = c;
        } else if (f.stage == 1) {
            f.left = ret;
            f.stage = 2;
            Frame c{f.off + f.n2, f.n - f.n2, 0, f.mid, f.hi, 0, 0, 0.0};
            st[sp++] = c;
        } else {
            ret = f.left + ret;
            sp--;
        }
    }
    return ret;
}

// The same sum as pairwise_sparse, for one wave: the m nonzeros' leaves of numpy's split tree
// (blocks of <= 128 elements; halving split rounded down to a multiple of 8) are found by
// the lanes in parallel (path bits + depth per nonzero), each leaf is summed by leaf_sum,
// and the leaves are combined in tree order by operator-precedence evaluation on the depth
// of each adjacent pair's lowest common split (the first differing path bit): O(m) serial
// steps instead of a walk over every split node.  Scratch (LDS, one wave): path[m], dep[m]
// ints, vals/ops stacks of AP_STACK entries.  Returns the sum on lane 0.
constexpr int AP_STACK = 34;

template <typename VAL>
__device__ double pairwise_tree_wave(const int* rk, VAL val, int m, int64_t n, uint32_t* path, int* dep,
                                     double* vals, int* ops) {
    const int lane = threadIdx.x & 63;
    for (int t = lane; t < m; t += 64) {
        int64_t off = 0, len = n;
        uint32_t pb = 0;
        int d = 0;
        while (len > 128) {
            int64_t n2 = len / 2;
            n2 -= n2 % 8;
            if ((int64_t)rk[t] - off < n2) len = n2;
            else { off += n2; len -= n2; pb |= 1u << d; }
            d++;
        }
        path[t] = pb;
        dep[t] = d;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    double res = 0.0;
    if (lane == 0) {
        int sp = 0, op = 0;
        int t = 0;
        while (t < m) {
            // leaf group [t, u): same path and depth
            int u = t + 1;
            while (u < m && path[u] == path[t] && dep[u] == dep[t]) u++;
            int64_t off = 0, len = n;
            for (int d = 0; d < dep[t]; d++) {  // the leaf's [off, off + len)
                int64_t n2 = len / 2;
                n2 -= n2 % 8;
                if ((path[t] >> d) & 1u) { off += n2; len -= n2; } else len = n2;
            }
            const double v = leaf_sum([&](int k) { return (int64_t)rk[k]; }, val, t, u, off, len);
            if (t > 0) {
                const int c = __builtin_ctz(path[t - 1] ^ path[t]);  // depth of the split between the leaves
                while (op > 0 && ops[op - 1] > c) {
                    const double b = vals[--sp];
                    vals[sp - 1] = vals[sp - 1] + b;
                    op--;
                }
                ops[op++] = c;
            }
            vals[sp++] = v;
            t = u;
        }
        while (op > 0) {
            const double b = vals[--sp];
            vals[sp - 1] = vals[sp - 1] + b;
            op--;
        }
        res = vals[0];
    }
    return res;
}

// pairwise_tree_wave's sum for m <= 64 with the leaves combined lane-parallel: lane t < m holds
// rk[t] (rk_l; rk is the same array in LDS, read for leaves holding several nonzeros).  Each
// leaf group's first lane sums its leaf (one nonzero: the value itself, x + zeros == x; more:
// leaf_sum over the group), then the splits are applied deepest first: at depth D every
// segment whose left boundary is a depth-D split adds itself into the segment on its left.
// Two depth-D boundaries never border the same segment (a shallower split lies between
// them), so this is pairwise_tree_wave's precedence evaluation step for step — the same
// additions, bit-identical — in (tree depth) wave steps instead of a serial chain over the
// leaves (that chain, even in registers, was ~27 % of a Market query:
// profiles/r02/eval_rows_phase_stamps.txt).
template <typename VAL>
__device__ double pairwise_tree_par(int rk_l, const int* rk, VAL val, int m, int64_t n) {
    const int lane = threadIdx.x & 63;
    const bool live = lane < m;
    uint32_t pb = 0;
    int d = 0;
    if (live) {
        int64_t off = 0, len = n;
        while (len > 128) {
            int64_t n2 = len / 2;
            n2 -= n2 % 8;
            if ((int64_t)rk_l - off < n2) len = n2;
            else { off += n2; len -= n2; pb |= 1u << d; }
            d++;
        }
    }
    const uint32_t ppb = (uint32_t)__shfl_up((int)pb, 1, 64);
    const int pd = __shfl_up(d, 1, 64);
    const bool head = live && (lane == 0 || ppb != pb || pd != d);
    const uint64_t heads = __ballot(head);
    double s = 0.0;
    int c = -1;  // depth of the split between the previous leaf and this one
    if (head) {
        const uint64_t above = (heads >> lane) >> 1;
        const int u = above ? lane + 1 + __builtin_ctzll(above) : m;
        if (u == lane + 1) {
            s = val(lane, rk_l);
        } else {
            int64_t off = 0, len = n;
            for (int e = 0; e < d; e++) {
                int64_t n2 = len / 2;
                n2 -= n2 % 8;
                if ((pb >> e) & 1u) { off += n2; len -= n2; } else len = n2;
            }
            s = leaf_sum([&](int k) { return (int64_t)rk[k]; }, [&](int k) { return val(k, rk[k]); }, lane, u, off,
                         len);
        }
        if (lane > 0) c = __builtin_ctz(ppb ^ pb);
    }
    int maxc = c;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const int t = __shfl_xor(maxc, o, 64);
        maxc = t > maxc ? t : maxc;
    }
    uint64_t act = heads;
    for (int D = maxc; D >= 0; D--) {
        const bool on = (act >> lane) & 1;
        const uint64_t mrg = __ballot(on && c == D);
        if (!mrg) continue;
        const uint64_t nxt = lane < 63 ? act >> (lane + 1) : 0;
        const int R = nxt ? lane + 1 + __builtin_ctzll(nxt) : lane;
        const double sr = __shfl(s, R, 64);
        if (on && nxt && ((mrg >> R) & 1)) s = s + sr;
        act &= ~mrg;
    }
    return __shfl(s, 0, 64);
}

// Per query (evaluate.py:40-80): positives = gallery items with the query's pid and another
// camera, junk = same pid and same camera (removed, :55-56), everything else a kept
// negative.  With the positives sorted by (distance, index) — np.argsort(kind="stable") —
// the rank of positive k among the kept items is
//     rank_k = #{all j : key_j < key_pk} - #{junk i : key_i < key_pk},
// so one pass over the distance row that bins EVERY item by how many positives precede it
// (b(j) = #{p : key_p < key_j}; rank_k + 1 + junk_before(k) = sum_{t <= k} hist[t]) gives all
// ranks; AP = numpy's pairwise sum of (k+1)/(rank_k+1) at positions rank_k over the kept
// length, / m (:73-79); first = rank_0 (the CMC step, :65-68).
//
// Gallery labels packed once per eval_rows call: when the gallery pids span < 65535 values
// (every ReID benchmark), pid - min as uint16 (padded to a multiple of 8 with 0xFFFF), so
// each query's label pass reads 2 B per item instead of 8 (it is L2 traffic repeated by
// every query).  Otherwise the kernel reads the int64 pids.
struct EvLabels {
    int64_t lo, hi;  // min / max gallery pid, biased to unsigned order for the atomics
};

__device__ __forceinline__ uint64_t ord64(int64_t v) { return (uint64_t)v ^ 0x8000000000000000ull; }
__device__ __forceinline__ int64_t unord64(uint64_t v) { return (int64_t)(v ^ 0x8000000000000000ull); }

__global__ void ev_minmax_init_kernel(unsigned long long* mm, int32_t* overflow) {
    mm[0] = ~0ull;
    mm[1] = 0ull;
    mm[2] = 0ull;  // eval_rows_kernel's arrival counter and huge-query count
    mm[3] = 0ull;  // "a query was deferred to eval_rows_kernel"
    *overflow = 0;
}

// min / max and the uint16 packing in ONE workgroup for galleries up to EV_PREP1_MAX (every
// ReID benchmark): one launch instead of three (each ~4-7 us at Market size, the kernel
// itself ~130 us).  Same outputs as ev_minmax_init/ev_minmax/ev_pack.
constexpr int64_t EV_PREP1_MAX = 1 << 18;

__global__ __launch_bounds__(1024) void ev_prep1_kernel(const int64_t* __restrict__ gp, int64_t G, int64_t G8,
                                                        unsigned long long* __restrict__ mm, uint16_t* __restrict__ pk,
                                                        int32_t* __restrict__ overflow) {
    __shared__ uint64_t slo[16], shi[16];
    const int tid = threadIdx.x;
    // 8 loads in flight per thread (a past-the-end item re-reads the last label: no effect on
    // min / max)
    constexpr int U = 8;
    uint64_t lo = ~0ull, hi = 0;
    for (int64_t j0 = 0; j0 < G; j0 += 1024 * U) {
        int64_t v[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int64_t j = j0 + u * 1024 + tid;
            v[u] = gp[j < G ? j : G - 1];
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint64_t o = ord64(v[u]);
            lo = o < lo ? o : lo;
            hi = o > hi ? o : hi;
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        const uint64_t a = __shfl_xor(lo, off, 64), b = __shfl_xor(hi, off, 64);
        lo = a < lo ? a : lo;
        hi = b > hi ? b : hi;
    }
    if ((tid & 63) == 0) { slo[tid >> 6] = lo; shi[tid >> 6] = hi; }
    __syncthreads();
    lo = slo[0];
    hi = shi[0];
    for (int w = 1; w < 16; w++) {
        lo = slo[w] < lo ? slo[w] : lo;
        hi = shi[w] > hi ? shi[w] : hi;
    }
    if (tid == 0) { mm[0] = lo; mm[1] = hi; mm[2] = 0ull; mm[3] = 0ull; *overflow = 0; }
    const int64_t plo = unord64(lo), phi = unord64(hi);
    if ((uint64_t)(phi - plo) >= 0xFFFFull) return;  // wide pid range: the int64 path
    for (int64_t j0 = 0; j0 < G8; j0 += 1024 * U) {
        int64_t v[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int64_t j = j0 + u * 1024 + tid;
            v[u] = gp[j < G ? j : G - 1];
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int64_t j = j0 + u * 1024 + tid;
            if (j < G8) pk[j] = j < G ? (uint16_t)(v[u] - plo) : (uint16_t)0xFFFF;
        }
    }
}

__global__ __launch_bounds__(256) void ev_minmax_kernel(const int64_t* __restrict__ gp, int64_t G,
                                                        unsigned long long* mm) {
    uint64_t lo = ~0ull, hi = 0;
    for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < G; j += (int64_t)gridDim.x * 256) {
        const uint64_t o = ord64(gp[j]);
        lo = o < lo ? o : lo;
        hi = o > hi ? o : hi;
    }
    for (int off = 32; off > 0; off >>= 1) {
        const uint64_t a = __shfl_xor(lo, off, 64), b = __shfl_xor(hi, off, 64);
        lo = a < lo ? a : lo;
        hi = b > hi ? b : hi;
    }
    if ((threadIdx.x & 63) == 0) {
        atomicMin(&mm[0], (unsigned long long)lo);
        atomicMax(&mm[1], (unsigned long long)hi);
    }
}

__global__ void ev_pack_kernel(const int64_t* __restrict__ gp, int64_t G, int64_t G8,
                               const unsigned long long* __restrict__ mm, uint16_t* __restrict__ pk) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= G8) return;
    const int64_t lo = unord64(mm[0]), hi = unord64(mm[1]);
    if ((uint64_t)(hi - lo) >= 0xFFFFull) return;  // wide pid range: the int64 path
    pk[j] = j < G ? (uint16_t)(gp[j] - lo) : (uint16_t)0xFFFF;
}

// eval_rows_wg_kernel: one 256-thread workgroup (4 waves) per query, ~17 KiB of LDS, 8
// workgroups per CU.  Pass 1 streams the gallery labels (uint16-packed, L2-resident: every
// query reads the same lines) and compacts the indices of the query's pid (ballot + one LDS
// atomic per wave and hit); their cameras and distances then come in ONE round trip and
// split them into positives and junk; the positives are bitonic-sorted in LDS.  Pass 2 reads
// the distance row once (16-byte loads after a scalar head to 16-byte alignment), skipping
// items beyond the last positive, and bins the rest into an LDS histogram through a bucket
// table of the positives (no per-item binary search: that search was 2/3 of the kernel).
// Wave 0 scans the histogram into ranks and sums the AP lane-parallel.  Queries with more
// than EVW_MAXP positives or EVW_MAXJ junk items are left to eval_rows_kernel (valid = 2).
// Per-phase cycle stamps: profiles/r02/eval_rows_phase_stamps.txt (-DEV_STAMPS build).
constexpr int EVW_MAXP = 512, EVW_MAXJ = 256, EVW_T = 1024;
#ifndef EV_PREFETCH
#define EV_PREFETCH 0
#endif
#ifndef EV_U1  // 16-byte label loads in flight per thread in the label pass
#define EV_U1 8
#endif

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8))) void eval_rows_wg_kernel(
    const float* __restrict__ dist, int64_t G, int64_t ld, const int64_t* __restrict__ qp,
    const int64_t* __restrict__ gp, const int64_t* __restrict__ qc, const int64_t* __restrict__ gc,
    const unsigned long long* __restrict__ mm, const uint16_t* __restrict__ pk, int32_t* __restrict__ valid,
    int64_t* __restrict__ first, double* __restrict__ ap, int64_t* __restrict__ nkept, int32_t* __restrict__ large) {
    __shared__ float pv[EVW_MAXP];
    __shared__ int pi[EVW_MAXP];
    __shared__ int hist[EVW_MAXP + 1];
    __shared__ float jv[EVW_MAXJ];
    __shared__ int ji[EVW_MAXJ];
    __shared__ int s_m, s_nj, s_ns;
    __shared__ double tvals[AP_STACK];
    __shared__ int tops[AP_STACK];
    // bucket t: {bits of the first positive in it (+inf when none), S[t] | 1 << 16 when it holds
    // two or more}; entry T = {+inf, m} closes the table (S[T] = m)
    __shared__ int2 bucket[EVW_T + 1];
    __shared__ int trash[256];  // one histogram slot per thread for the items not binned
    const int tid = threadIdx.x, lane = tid & 63;
#ifdef EV_STAMPS
    const uint64_t t0 = __builtin_amdgcn_s_memtime(), rt0 = __builtin_amdgcn_s_memrealtime();
    uint64_t t1 = 0, t2 = 0, t3 = 0;
#endif
    const int64_t q = blockIdx.x;
    const float* row = dist + q * ld;
    const int64_t qpid = qp[q], qcam = qc[q];
    const uint64_t below = (1ull << lane) - 1;
    int* sidx = (int*)bucket;  // same-pid gallery indices of pass 1 (the bucket table comes later)
    constexpr int SCAP = EVW_MAXP + EVW_MAXJ;
    // the distance pass's layout (16-byte loads after a scalar head) and its first chunk,
    // loaded now so its latency hides behind the label pass and the sort
    const int head = (int)(((16 - ((uintptr_t)row & 15)) & 15) >> 2);  // scalar items before 16-B alignment
    const int h = head < G ? head : (int)G;
    const int nv = (int)((G - h) >> 2);  // float4 groups (G < 2^31)
    const float4* r4 = (const float4*)(row + h);
    constexpr int U2 = 4;
    float4 v[U2];
    auto load_chunk = [&](int g0) {  // past the row's end: reload its last group, not binned
#pragma unroll
        for (int u = 0; u < U2; u++) {
            const int g = g0 + u * 256 + tid;
            v[u] = r4[g < nv ? g : nv - 1];
        }
    };
#if EV_PREFETCH
    if (nv > 0) load_chunk(0);
#endif
    if (tid == 0) { s_m = 0; s_nj = 0; s_ns = 0; }
    __syncthreads();
    // ---- pass 1: labels -> indices of the gallery items with the query's pid (ballot
    // compaction, one LDS atomic per wave and hit).  Every workgroup reads the same label
    // lines, so each starts at its own chunk.
    auto take = [&](bool same, int64_t j) {
        const uint64_t ms = __ballot(same);
        int base = 0;
        if (lane == 0) base = atomicAdd(&s_ns, __popcll(ms));
        base = __shfl(base, 0, 64);
        const int sl = base + __popcll(ms & below);
        if (same && sl < SCAP) sidx[sl] = (int)j;
    };
    const int64_t plo = unord64(mm[0]), phi = unord64(mm[1]);
    if ((uint64_t)(phi - plo) < 0xFFFFull) {  // packed uint16 labels, 8 per 16-byte load
        if (qpid >= plo && qpid <= phi) {
            const uint16_t key = (uint16_t)(qpid - plo);
            constexpr int U1 = EV_U1, CH = 2048 * U1;
            const int64_t nch = (G + CH - 1) / CH;
            const int64_t c0 = (q * 37) % nch;
            const int64_t n8 = (G + 7) / 8;
            for (int64_t c = 0; c < nch; c++) {
                int64_t v0 = ((c0 + c) % nch) * (CH / 8);
                uint4 w[U1];
#pragma unroll
                for (int u = 0; u < U1; u++) {
                    const int64_t v = v0 + u * 256 + tid;
                    w[u] = v < n8 ? ((const uint4*)pk)[v] : make_uint4(~0u, ~0u, ~0u, ~0u);
                }
                // 8 labels per lane tested at once: a 16-bit half of x = d ^ (key | key << 16)
                // is zero iff that label is the key (padding 0xFFFF never equals a key); one
                // ballot per 8 labels, the per-label ballots only where some lane hit
                const uint32_t kk = (uint32_t)key * 0x10001u;
#pragma unroll
                for (int u = 0; u < U1; u++) {
                    const int64_t jb = (v0 + u * 256 + tid) * 8;
                    const uint32_t d[4] = {w[u].x ^ kk, w[u].y ^ kk, w[u].z ^ kk, w[u].w ^ kk};
                    bool any = false;
#pragma unroll
                    for (int e = 0; e < 4; e++) any = any || (d[e] & 0xFFFFu) == 0u || (d[e] >> 16) == 0u;
                    if (!__ballot(any)) continue;
#pragma unroll
                    for (int e = 0; e < 8; e++) {
                        const bool same = ((d[e >> 1] >> (16 * (e & 1))) & 0xFFFFu) == 0u;
                        if (__ballot(same)) take(same, jb + e);
                    }
                }
            }
        }
    } else {
        constexpr int U1 = 4, CH = 256 * U1;
        const int64_t nch = (G + CH - 1) / CH;
        const int64_t c0 = (q * 37) % nch;
        for (int64_t c = 0; c < nch; c++) {
            const int64_t j0 = ((c0 + c) % nch) * CH;
            int64_t pid[U1];
#pragma unroll
            for (int u = 0; u < U1; u++) {
                const int64_t j = j0 + u * 256 + tid;
                pid[u] = j < G ? gp[j] : qpid + 1;
            }
#pragma unroll
            for (int u = 0; u < U1; u++) {
                const bool same = pid[u] == qpid;
                if (__ballot(same)) take(same, j0 + u * 256 + tid);
            }
        }
    }
    __syncthreads();
    const int ns = s_ns;
    // ---- split them into positives (other camera) and junk (same camera, removed,
    // evaluate.py:55-56), their cameras and distances loaded in one round trip
    if (ns <= SCAP) {
        for (int t = tid; t < ns; t += 256) {
            const int j = sidx[t];
            const int64_t cam = gc[j];
            const float v = row[j];
            if (cam == qcam) {
                const int sl = atomicAdd(&s_nj, 1);
                if (sl < EVW_MAXJ) { ji[sl] = j; jv[sl] = v; }
            } else {
                const int sl = atomicAdd(&s_m, 1);
                if (sl < EVW_MAXP) { pi[sl] = j; pv[sl] = v; }
            }
        }
    }
    __syncthreads();
    const int m = s_m, nj = s_nj;
#ifdef EV_STAMPS
    t1 = __builtin_amdgcn_s_memtime();
#endif
    if (ns > SCAP || m > EVW_MAXP || nj > EVW_MAXJ) {  // eval_rows_kernel (large lists) takes it
        if (tid == 0) {
            valid[q] = 2;
            *large = 1;
        }
        return;
    }
    if (tid == 0) nkept[q] = G - nj;
    if (m == 0) {
        if (tid == 0) { valid[q] = 0; first[q] = -1; ap[q] = 0.0; }
        return;
    }
    // ---- sort the positives by (value, index)
    int P = 1;
    while (P < m) P <<= 1;
    for (int t = m + tid; t < P; t += 256) {
        pv[t] = __builtin_inff();
        pi[t] = 0x7fffffff;
    }
    for (int t = tid; t <= m; t += 256) hist[t] = 0;
    __syncthreads();
    bitonic_sort_kv(pv, pi, P);
    // ---- pass 2: bin every item of the row by the number of positives before it.  A
    // bucket table narrows each item's candidates: t(x) = clamp(floor((x - v_0) * T /
    // (v_last - v_0)), 0, T-1) is monotone in x (the same float operations for every x), so
    // positives in buckets below t(x) are all smaller, those above all larger, and only the
    // positives of bucket t(x) need the exact (value, index) compare.  The table entry carries
    // the bucket's first positive value: with at most one positive in the bucket and no tie
    // with it, b = S[t] + (v_first < x) — branch-free, one 8-byte LDS read per item; buckets
    // of two or more positives and exact ties take the (value, index) walk, per wave only when
    // some lane needs it.
    const float lv = pv[m - 1];
    const int li = pi[m - 1];
    const float v0 = pv[0];
    const int T = 8 * P < EVW_T ? (8 * P > 64 ? 8 * P : 64) : EVW_T;  // ~8 buckets per positive
    // t(x) = floor(med3(x * scale - v_0 * scale, 0, T-1)): one fma, one med3, one convert
    // per item; when the positives tie (scale inf / NaN) every item goes to bucket 0 and the
    // exact compares decide
    float scale = (float)T / (lv - v0);
    if (!(scale <= 3.0e38f)) scale = 0.0f;
    const float c0 = -v0 * scale, tmax = (float)(T - 1);
    auto bucket_of = [&](float x) {  // med3 clamps to [0, T-1] (NaN to 0 or T-1), truncation floors
        return (int)__builtin_amdgcn_fmed3f(__builtin_fmaf(x, scale, c0), 0.0f, tmax);
    };
    constexpr int MULTI = 1 << 16;
    for (int t = tid; t <= T; t += 256) {  // S[t] = #{k : t(pv_k) < t}; n_t positives in bucket t
        int lo = m, n = 0;
        if (t < T) {
            lo = 0;
            int hi = m;
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (bucket_of(pv[mid]) < t) lo = mid + 1; else hi = mid;
            }
            int lo2 = lo, hi2 = m;
            while (lo2 < hi2) {
                const int mid = (lo2 + hi2) >> 1;
                if (bucket_of(pv[mid]) <= t) lo2 = mid + 1; else hi2 = mid;
            }
            n = lo2 - lo;
        }
        bucket[t] = make_int2(n > 0 ? __float_as_int(pv[lo]) : 0x7f800000, lo | (n > 1 ? MULTI : 0));
    }
    __syncthreads();
#ifdef EV_STAMPS
    t2 = __builtin_amdgcn_s_memtime();
#endif
    // b for an item of bucket t with entry e: the exact (value, index) walk over the bucket
    auto walk = [&](int t, int2 e, float v, int j) {
        int b = e.y & 0xFFFF;
        const int end = bucket[t + 1].y & 0xFFFF;
        while (b < end && key_less(pv[b], pi[b], v, j)) b++;
        return b;
    };
    auto bin = [&](float v, int j) {
        // after the last positive (b = m, not needed); NaN sorts last (np.argsort):
        // key_less(lv, li, v, j) || v != v, with the NaN test folded into !(v <= lv)
        if (!(v <= lv) || (v == lv && j > li)) return;
        const int t = bucket_of(v);
        atomicAdd(&hist[walk(t, bucket[t], v, j)], 1);
    };
    if (tid < h) bin(row[tid], tid);
    int* const mytrash = &trash[tid];
    for (int g0 = 0; g0 < nv; g0 += 256 * U2) {
        if (!EV_PREFETCH || g0 > 0) load_chunk(g0);
#pragma unroll
        for (int u = 0; u < U2; u++) {
            const int g = g0 + u * 256 + tid;
            const float x[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
            int tb[4];
            bool ok[4];
#pragma unroll
            for (int k = 0; k < 4; k++) {
                // items after the last positive are not needed (b = m); NaN sorts last
                // (np.argsort) and fails x <= lv.  An item tied with the last positive's value
                // but after it (x == lv, j > li) is binned: it gets b = m, a count in hist[m]
                // that no rank reads
                ok[k] = (g < nv) & (x[k] <= lv);
                tb[k] = bucket_of(x[k]);
            }
            int2 se[4];
#pragma unroll
            for (int k = 0; k < 4; k++) se[k] = bucket[tb[k]];
            int b[4];
            bool sl[4], slow = false;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const float vf = __int_as_float(se[k].x);
                b[k] = (se[k].y & 0xFFFF) + (vf < x[k] ? 1 : 0);
                sl[k] = ok[k] & ((se[k].y >= MULTI) | (vf == x[k]));
                slow = slow | sl[k];
            }
            if (__ballot(slow)) {
#pragma unroll
                for (int k = 0; k < 4; k++)
                    if (sl[k]) b[k] = walk(tb[k], se[k], x[k], h + g * 4 + k);
            }
#pragma unroll
            for (int k = 0; k < 4; k++) atomicAdd(ok[k] ? &hist[b[k]] : mytrash, 1);
        }
    }
    for (int64_t j = h + (int64_t)nv * 4 + tid; j < G; j += 256) bin(row[j], (int)j);
    __syncthreads();
#ifdef EV_STAMPS
    t3 = __builtin_amdgcn_s_memtime();
#endif
    // ---- ranks (wave 0): inclusive scan of hist, minus the item itself and the junk before it
    if (tid < 64) {
        int carry = 0;
        for (int c0 = 0; c0 < m; c0 += 64) {
            const int k = c0 + lane;
            int v = k < m ? hist[k] : 0;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const int t = __shfl_up(v, o, 64);
                if (lane >= o) v += t;
            }
            const int incl = v + carry;
            carry = __shfl(incl, 63, 64);
            if (k < m) {
                const float pvk = pv[k];
                const int pik = pi[k];
                int jb = 0;
                for (int t = 0; t < nj; t++) jb += key_less(jv[t], ji[t], pvk, pik);
                hist[k] = incl - 1 - jb;  // rank_k (0-based position among the kept items)
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        const int* rk = hist;
        const double sum =
            m <= 64 ? pairwise_tree_par(lane < m ? rk[lane] : 0, rk,
                                        [](int t, int r) { return (double)(t + 1) / (double)(r + 1); }, m, G - nj)
                    : pairwise_tree_wave(rk, [&](int t) { return (double)(t + 1) / (double)(rk[t] + 1); }, m, G - nj,
                                         (uint32_t*)pv, pi, tvals, tops);  // pv / pi are free now
        if (lane == 0) {
            valid[q] = 1;
            first[q] = rk[0];
            ap[q] = sum / (double)m;
#ifdef EV_STAMPS
            const uint64_t t4 = __builtin_amdgcn_s_memtime();
            first[q] = (int64_t)((t1 - t0) | ((t2 - t1) << 32));
            nkept[q] = (int64_t)((t3 - t2) | ((t4 - t3) << 32));
            ap[q] = (double)rt0;
#endif
        }
    }
}

constexpr int EV_MAXP = 2048;

// Fallback for the queries eval_rows_wg_kernel left (valid == 2: more than EVW_MAXP
// positives or EVW_MAXJ junk items): one workgroup per query, up to EV_MAXP positives in
// LDS.  Positives are collected and sorted; every other kept gallery item is binned by how
// many positives precede it (binary search).  A query with more positives than that is
// marked valid = 3 and evaluated by the kernel's LAST workgroup to finish, with the same
// code on scratch arrays in the call's workspace sized for the whole gallery (EvScratch):
// no capacity limit, as in the reference.
struct EvLargeLds {
    float pv[EV_MAXP];
    int pi[EV_MAXP];
    int hist[EV_MAXP + 1];
    int64_t rk[EV_MAXP];
    double rv[EV_MAXP];
    int s_m, s_junk;
    PwFrame pw[PW_DEPTH];
};

struct EvScratch {  // arrays of the large-list evaluation (LDS, or global memory)
    float* pv;
    int* pi;
    int* hist;
    int64_t* rk;
    double* rv;
    int64_t cap;  // positives the arrays hold (pv / pi hold pow2_ceil(cap))
};

// returns false (and sets nothing) when the query has more than S.cap positives
__device__ bool eval_row_large(int64_t q, const float* __restrict__ dist, int64_t G, int64_t ld,
                               const int64_t* __restrict__ qp, const int64_t* __restrict__ gp,
                               const int64_t* __restrict__ qc, const int64_t* __restrict__ gc,
                               int32_t* __restrict__ valid, int64_t* __restrict__ first, double* __restrict__ ap,
                               int64_t* __restrict__ nkept, const EvScratch& S, EvLargeLds& L) {
    float* pv = S.pv;
    int* pi = S.pi;
    int* hist = S.hist;
    int64_t* rk = S.rk;
    double* rv = S.rv;
    int& s_m = L.s_m;
    int& s_junk = L.s_junk;
    PwFrame* pw = L.pw;
    const float* row = dist + q * ld;
    const int64_t qpid = qp[q], qcam = qc[q];
    if (threadIdx.x == 0) { s_m = 0; s_junk = 0; }
    __syncthreads();
    for (int64_t j = threadIdx.x; j < G; j += blockDim.x) {
        if (gp[j] == qpid) {
            if (gc[j] == qcam) atomicAdd(&s_junk, 1);
            else {
                int p = atomicAdd(&s_m, 1);
                if (p < S.cap) { pv[p] = row[j]; pi[p] = (int)j; }
            }
        }
    }
    __syncthreads();
    const int m = s_m;
    if (m > S.cap) return false;
    const int P = pow2_ceil(m < 2 ? 2 : m);
    for (int t = m + threadIdx.x; t < P; t += blockDim.x) { pv[t] = __builtin_inff(); pi[t] = 0x7fffffff; }
    for (int t = threadIdx.x; t <= m; t += blockDim.x) hist[t] = 0;
    __syncthreads();
    bitonic_sort_kv(pv, pi, P);
    for (int64_t j = threadIdx.x; j < G; j += blockDim.x) {
        if (gp[j] == qpid) continue;  // positives counted separately, junk removed
        const float v = row[j];
        int lo = 0, hi = m;
        while (lo < hi) {
            int mid = (lo + hi) >> 1;
            if (key_less(pv[mid], pi[mid], v, (int)j)) lo = mid + 1; else hi = mid;
        }
        if (lo < m) atomicAdd(&hist[lo], 1);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const int64_t n = G - s_junk;
        nkept[q] = n;
        valid[q] = 1;
        int64_t cum = 0;
        for (int k = 0; k < m; k++) {
            cum += hist[k];
            rk[k] = k + cum;
            rv[k] = (double)(k + 1) / (double)(rk[k] + 1);
        }
        first[q] = rk[0];
        ap[q] = pairwise_sparse([&](int t) { return rk[t]; }, [&](int t) { return rv[t]; }, m, n, pw) / (double)m;
    }
    __syncthreads();
    return true;
}

// Grid-stride over the queries (a few workgroups per CU instead of one launch-slot per query);
// the last workgroup to finish takes the queries marked valid = 3.  A workgroup that marked
// one counts it (hugecount) and issues a release fence before its arrival; the last arrival
// issues an acquire fence and, only when the count is non-zero, scans valid[] in parallel —
// nothing of this runs unless eval_rows_wg_kernel deferred a query (*large).
__global__ __launch_bounds__(256) void eval_rows_kernel(
    const float* __restrict__ dist, int64_t Q, int64_t G, int64_t ld, const int64_t* __restrict__ qp,
    const int64_t* __restrict__ gp, const int64_t* __restrict__ qc, const int64_t* __restrict__ gc,
    int32_t* __restrict__ valid, int64_t* __restrict__ first, double* __restrict__ ap,
    int64_t* __restrict__ nkept, const int32_t* __restrict__ large, unsigned int* __restrict__ arrivals,
    unsigned int* __restrict__ hugecount, EvScratch huge) {
    if (*large == 0) return;  // no query left for this kernel (the common case: one load per workgroup)
    __shared__ EvLargeLds L;
    __shared__ int s_last, s_mark;
    __shared__ unsigned int s_cnt;
    const EvScratch lds{L.pv, L.pi, L.hist, L.rk, L.rv, EV_MAXP};
    if (threadIdx.x == 0) s_mark = 0;
    __syncthreads();
    for (int64_t q = blockIdx.x; q < Q; q += gridDim.x) {
        if (valid[q] != 2) continue;  // uniform per workgroup
        if (!eval_row_large(q, dist, G, ld, qp, gp, qc, gc, valid, first, ap, nkept, lds, L) && threadIdx.x == 0) {
            valid[q] = 3;
            s_mark = 1;
            atomicAdd(hugecount, 1u);
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        if (s_mark) __threadfence();
        const unsigned int prev = __hip_atomic_fetch_add(arrivals, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_last = prev == gridDim.x - 1;
        s_cnt = 0;
        if (s_last) {
            __threadfence();
            s_cnt = __hip_atomic_load(hugecount, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    __syncthreads();
    if (!s_last || s_cnt == 0) return;
    __shared__ int flag[256];
    for (int64_t q0 = 0; q0 < Q; q0 += blockDim.x) {
        const int64_t q = q0 + threadIdx.x;
        const bool h = q < Q && valid[q] == 3;
        flag[threadIdx.x] = h;
        if (!__syncthreads_or(h)) continue;
        for (int t = 0; t < (int)blockDim.x; t++)
            if (flag[t]) eval_row_large(q0 + t, dist, G, ld, qp, gp, qc, gc, valid, first, ap, nkept, huge, L);
        __syncthreads();
    }
}

// The pair bound's constants for D-dimensional features (fp16-rounded operands, fp32 MFMA
// accumulation; the derivation is in rank_select_kernel's description of the bound).
void rank_select_consts(int D, float c[3]) {
    const double c_rel = 2.0 * (0x1p-10 + 0x1p-22 + 2.02 * D * 0x1p-24) + 2.02 * 0x1p-23;
    const double c_abs = 2.01 * 0x1p-25 * std::sqrt((double)D);
    const double c_d = D * 0x1p-49;
    c[0] = (float)(c_rel * (1.0 + 0x1p-20));
    c[1] = (float)(c_abs * (1.0 + 0x1p-20));
    c[2] = (float)(c_d * (1.0 + 0x1p-20));
}

// max over the items of the norms (out2[0]) and squared norms (out2[1]); fmaxf skips NaN (a NaN
// norm makes its bounds NaN, which sends the rows to the exact path)
__global__ __launch_bounds__(1024) void norm_max_kernel(const float* __restrict__ sqn, const float* __restrict__ nrm,
                                                        int64_t N, float* __restrict__ out2) {
    __shared__ float red[2][16];
    float a = 0.0f, b = 0.0f;
    for (int64_t j = threadIdx.x; j < N; j += blockDim.x) {
        a = fmaxf(a, nrm[j]);
        b = fmaxf(b, sqn[j]);
    }
    a = wave_max(a);
    b = wave_max(b);
    if ((threadIdx.x & 63) == 0) {
        red[0][threadIdx.x >> 6] = a;
        red[1][threadIdx.x >> 6] = b;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < 16; w++) {
            a = fmaxf(a, red[0][w]);
            b = fmaxf(b, red[1][w]);
        }
        out2[0] = a;
        out2[1] = b;
    }
}

int norm_max_launch(const float* sqn, const float* nrm, int64_t N, float* out2, hipStream_t s) {
    RM_REQUIRE(N > 0 && sqn && nrm && out2, "norm_max: bad arguments");
    hipLaunchKernelGGL(norm_max_kernel, dim3(1), dim3(1024), 0, s, sqn, nrm, N, out2);
    RM_LAUNCHED();
    return OK;
}

// rank_select_kernel over rows [row0, row0 + rows) of the pre-filter bounds `dot` ([rows][ldd]
// fp32 hi, ldd >= N, the EPI_RRHI GEMM), nmax2 = norm_max_kernel's maxima.
int rank_select_launch(float* dot, int64_t ldd, const float* feat, int64_t ldf, int D, const float* sqn,
                       const float* nrm, const float* nmax2, int64_t row0, int64_t rows, int64_t N, int K,
                       int32_t* rank_out, float* rowmax_out, int32_t* need, hipStream_t s) {
    RM_REQUIRE(K >= 1 && K <= 64 && K <= N && ldd >= N && ldd % 4 == 0 && rows >= 0 && nmax2 &&
                   ((uintptr_t)dot & 15) == 0,
               "rank_select: bad arguments");
    if (rows == 0) return OK;
    float c[3];
    rank_select_consts(D, c);
#ifndef RS_SINGLE_PASS
#define RS_SINGLE_PASS 1
#endif
    hipLaunchKernelGGL(RS_SINGLE_PASS ? rank_select1_kernel : rank_select_kernel, dim3((unsigned)rows), dim3(256), 0,
                       s, dot, ldd, feat, ldf, D, sqn, nrm, row0, N, K, c[0], c[1], c[2], nmax2, rank_out, rowmax_out,
                       need);
    RM_LAUNCHED();
    return OK;
}

int feat16_launch(const float* x, int64_t N, int64_t D, int64_t ldx, void* y, int64_t Np, int64_t Dp,
                  int32_t* range_ok, hipStream_t s) {
    RM_REQUIRE(N > 0 && D > 0 && ldx >= D && Np >= N && Dp >= D && range_ok, "feat16: bad arguments");
    hipLaunchKernelGGL(feat16_kernel, dim3((unsigned)ceil_div(Np * Dp, 256)), dim3(256), 0, s, x, N, D, ldx,
                       (_Float16*)y, Np, Dp, range_ok);
    RM_LAUNCHED();
    return OK;
}

int topk_launch(const float* x, int64_t rows, int64_t cols, int64_t ldx, const float* row_div, int K,
                int32_t* out_idx, float* out_val, int64_t ldo, hipStream_t s) {
    RM_REQUIRE(rows >= 0 && cols > 0 && ldx >= cols && K > 0 && K <= cols && ldo >= K,
               "topk_rows: need 0 < k <= cols, ldo >= k");
    RM_REQUIRE(cols < 0x7fffffff, "topk_rows: cols must fit int32");
    if (rows == 0) return OK;
    hipLaunchKernelGGL(topk_rows_kernel, dim3((unsigned)rows), dim3(256), 0, s, x, cols, ldx, row_div, K, out_idx,
                       out_val, ldo);
    RM_LAUNCHED();
    return OK;
}

int distmat_impl(bool cosine, const float* q, int64_t Q, int64_t ldq, const float* g, int64_t G, int64_t ldg,
                 int64_t D, float* out, int64_t ldo, float* ws, void* stream, int variant = 0);

int distmat_launch(const float* q, int64_t Q, int64_t ldq, const float* g, int64_t G, int64_t ldg, int64_t D,
                   float* out, int64_t ldo, float* ws, hipStream_t s) {
    return distmat_impl(false, q, Q, ldq, g, G, ldg, D, out, ldo, ws, s);
}

// Euclidean distance with precomputed squared row norms qq[Q], gg[G] (row_sqnorm_kernel).
int distmat_pre_launch(const float* q, int64_t Q, int64_t ldq, const float* g, int64_t G, int64_t ldg, int64_t D,
                       const float* qq, const float* gg, float* out, int64_t ldo, hipStream_t s) {
    RM_REQUIRE(Q >= 0 && G >= 0 && D > 0 && ldq >= D && ldg >= D && ldo >= G && qq && gg, "distmat: bad shape");
    if (Q == 0 || G == 0) return OK;
    dim3 grid(ceil_div(G, DM_BN), ceil_div(Q, DM_BM));
    RM_REQUIRE(grid.y <= 65535, "distmat: too many query rows for one launch");
    if (dm2_ok(q, ldq, g, ldg, D))
        hipLaunchKernelGGL(distmat2_f32_kernel<false>, dim3((unsigned)((int64_t)grid.x * grid.y)), dim3(256), 0, s, q, g,
                           qq, gg, Q, G, D, ldq, ldg, out, ldo);
    else
        hipLaunchKernelGGL(distmat_f32_kernel<false>, grid, dim3(256), 0, s, q, g, qq, gg, Q, G, D, ldq, ldg, out, ldo);
    RM_LAUNCHED();
    return OK;
}

}  // namespace reidmi

using namespace reidmi;

REIDMI_API int reidmi_row_sqnorm_f32(const float* x, int64_t n, int64_t d, int64_t ldx, float* out, void* stream) {
    RM_REQUIRE(n >= 0 && d >= 0 && ldx >= d, "row_sqnorm: bad shape");
    if (n == 0) return OK;
    rows_sqnorm_launch(x, n, d, ldx, out, (hipStream_t)stream);
    RM_LAUNCHED();
    return OK;
}

REIDMI_API int reidmi_l2norm_f32(const float* x, int64_t n, int64_t d, int64_t ldx, float* y, int64_t ldy,
                                 float* ws, void* stream) {
    RM_REQUIRE(n >= 0 && d > 0 && ldx >= d && ldy >= d && ws != nullptr, "l2norm: bad shape or workspace");
    if (n == 0) return OK;
    hipStream_t s = (hipStream_t)stream;
    rows_sqnorm_launch(x, n, d, ldx, ws, s);
    RM_LAUNCHED();
    hipLaunchKernelGGL(row_scale_kernel, dim3((unsigned)n), dim3(256), 0, s, x, ws, d, ldx, y, ldy);
    RM_LAUNCHED();
    return OK;
}

int reidmi::distmat_impl(bool cosine, const float* q, int64_t Q, int64_t ldq, const float* g, int64_t G,
                        int64_t ldg, int64_t D, float* out, int64_t ldo, float* ws, void* stream, int variant) {
    RM_REQUIRE(variant == 0 || variant == 1, "distmat variant: 0 auto, 1 single-stage");
    RM_REQUIRE(Q >= 0 && G >= 0 && D > 0 && ldq >= D && ldg >= D && ldo >= G, "distmat: bad shape");
    RM_REQUIRE(ws != nullptr, "distmat: workspace (Q+G floats) required");
    if (Q == 0 || G == 0) return OK;
    hipStream_t s = (hipStream_t)stream;
    float* qq = ws;
    float* gg = ws + Q;
    rows_sqnorm_launch(q, Q, D, ldq, qq, s);
    RM_LAUNCHED();
    rows_sqnorm_launch(g, G, D, ldg, gg, s);
    RM_LAUNCHED();
    dim3 grid(ceil_div(G, DM_BN), ceil_div(Q, DM_BM));
    RM_REQUIRE(grid.y <= 65535, "distmat: too many query rows for one launch");
    const bool v2 = dm2_ok(q, ldq, g, ldg, D) && variant != 1;
    const dim3 grid1((unsigned)((int64_t)grid.x * grid.y));
    if (cosine) {
        if (v2)
            hipLaunchKernelGGL(distmat2_f32_kernel<true>, grid1, dim3(256), 0, s, q, g, qq, gg, Q, G, D, ldq, ldg, out, ldo);
        else
            hipLaunchKernelGGL(distmat_f32_kernel<true>, grid, dim3(256), 0, s, q, g, qq, gg, Q, G, D, ldq, ldg, out, ldo);
    } else {
        if (v2)
            hipLaunchKernelGGL(distmat2_f32_kernel<false>, grid1, dim3(256), 0, s, q, g, qq, gg, Q, G, D, ldq, ldg, out,
                               ldo);
        else
            hipLaunchKernelGGL(distmat_f32_kernel<false>, grid, dim3(256), 0, s, q, g, qq, gg, Q, G, D, ldq, ldg, out, ldo);
    }
    RM_LAUNCHED();
    return OK;
}

REIDMI_API int reidmi_distmat_f32(const float* q, int64_t Q, int64_t ldq, const float* g, int64_t G, int64_t ldg,
                                  int64_t D, float* out, int64_t ldo, float* ws, void* stream) {
    return distmat_impl(false, q, Q, ldq, g, G, ldg, D, out, ldo, ws, stream);
}

#ifdef REIDMI_TOOLS
// Per-call kernel selection (tests / A-B timing; tools library, include/reidmi_tools.h):
// 0 = auto (pipelined when the operands allow), 1 = the single-stage kernel; the same MFMA
// chain per output (bit-identical).
REIDMI_API int reidmi_distmat_f32_variant(const float* q, int64_t Q, int64_t ldq, const float* g, int64_t G,
                                          int64_t ldg, int64_t D, float* out, int64_t ldo, float* ws, int variant,
                                          void* stream) {
    return distmat_impl(false, q, Q, ldq, g, G, ldg, D, out, ldo, ws, stream, variant);
}
#endif

REIDMI_API int reidmi_cosine_f32(const float* q, int64_t Q, int64_t ldq, const float* g, int64_t G, int64_t ldg,
                                 int64_t D, float* out, int64_t ldo, float* ws, void* stream) {
    return distmat_impl(true, q, Q, ldq, g, G, ldg, D, out, ldo, ws, stream);
}

REIDMI_API int reidmi_topk_rows_f32(const float* x, int64_t rows, int64_t cols, int64_t ldx, const float* row_div,
                                    int k, int32_t* out_idx, float* out_val, int64_t ldo, void* stream) {
    return topk_launch(x, rows, cols, ldx, row_div, k, out_idx, out_val, ldo, (hipStream_t)stream);
}

// workspace: [0, 256) min/max + arrival counter | packed labels (G8 uint16) | large-list
// scratch for one query of up to G positives: pv, pi (pow2_ceil(G) each), hist (G + 1),
// rk, rv (G each)
static int64_t ev_pow2(int64_t G) {
    int64_t p = 2;
    while (p < G) p <<= 1;
    return p;
}
static int64_t ev_lab_bytes(int64_t G) { return ((G + 7) / 8 * 8) * 2; }
static int64_t ev_huge_off(int64_t G) { return (256 + ev_lab_bytes(G) + 15) / 16 * 16; }
static int64_t ev_ws_bytes(int64_t G) {
    const int64_t P2 = ev_pow2(G);
    return ev_huge_off(G) + P2 * 8 + ((G + 1) * 4 + 7) / 8 * 8 + G * 16;
}

REIDMI_API int64_t reidmi_eval_rows_workspace_bytes(int64_t G) { return G > 0 ? ev_ws_bytes(G) : -1; }

REIDMI_API int reidmi_eval_rows(const float* dist, int64_t Q, int64_t G, int64_t ldd, const int64_t* q_pids,
                                const int64_t* g_pids, const int64_t* q_cams, const int64_t* g_cams, int32_t* valid,
                                int64_t* first, double* ap, int64_t* nkept, int32_t* overflow, void* ws_,
                                int64_t ws_bytes, void* stream) {
    RM_REQUIRE(Q >= 0 && G > 0 && ldd >= G && G < 0x7fffffff, "eval_rows: bad shape");
    RM_REQUIRE(overflow != nullptr, "eval_rows: overflow flag pointer required");
    RM_REQUIRE(((uintptr_t)dist & 3) == 0, "eval_rows: dist must be 4-byte aligned");
    RM_REQUIRE(ws_ != nullptr && ((uintptr_t)ws_ & 15) == 0 && ws_bytes >= ev_ws_bytes(G),
               "eval_rows: workspace (reidmi_eval_rows_workspace_bytes, 16-byte aligned) required");
    if (Q == 0) return OK;
    RM_REQUIRE(Q < (1ll << 31), "eval_rows: too many queries");
    hipStream_t s = (hipStream_t)stream;
    unsigned long long* mm = (unsigned long long*)ws_;
    uint16_t* pk = (uint16_t*)((char*)ws_ + 256);
    const int64_t G8 = (G + 7) / 8 * 8;
    if (G <= EV_PREP1_MAX) {
        hipLaunchKernelGGL(ev_prep1_kernel, dim3(1), dim3(1024), 0, s, g_pids, G, G8, mm, pk, overflow);
        RM_LAUNCHED();
    } else {
        hipLaunchKernelGGL(ev_minmax_init_kernel, dim3(1), dim3(1), 0, s, mm, overflow);
        RM_LAUNCHED();
        hipLaunchKernelGGL(ev_minmax_kernel, dim3((unsigned)std::min<int64_t>(ceil_div(G, 256), 1024)), dim3(256), 0,
                           s, g_pids, G, mm);
        RM_LAUNCHED();
        hipLaunchKernelGGL(ev_pack_kernel, dim3(ceil_div(G8, 256)), dim3(256), 0, s, g_pids, G, G8,
                           (const unsigned long long*)mm, pk);
        RM_LAUNCHED();
    }
    hipLaunchKernelGGL(eval_rows_wg_kernel, dim3((unsigned)Q), dim3(256), 0, s, dist, G, ldd, q_pids, g_pids, q_cams,
                       g_cams, (const unsigned long long*)mm, (const uint16_t*)pk, valid, first, ap, nkept,
                       (int32_t*)(mm + 3));
    RM_LAUNCHED();
    EvScratch huge{};
    {
        char* h = (char*)ws_ + ev_huge_off(G);
        const int64_t P2 = ev_pow2(G);
        huge.pv = (float*)h;
        huge.pi = (int*)(h + P2 * 4);
        huge.hist = (int*)(h + P2 * 8);
        huge.rk = (int64_t*)(h + P2 * 8 + ((G + 1) * 4 + 7) / 8 * 8);
        huge.rv = (double*)((char*)huge.rk + G * 8);
        huge.cap = G;
    }
    hipLaunchKernelGGL(eval_rows_kernel, dim3((unsigned)std::min<int64_t>(Q, 512)), dim3(256), 0, s, dist, Q, G, ldd,
                       q_pids, g_pids, q_cams, g_cams, valid, first, ap, nkept, (const int32_t*)(mm + 3),
                       (unsigned int*)(mm + 2), (unsigned int*)(mm + 2) + 1, huge);
    RM_LAUNCHED();
    return OK;
}
