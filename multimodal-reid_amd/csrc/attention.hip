// attention.hip — fused multi-head self-attention for the CLIP encoders (gfx950).
//
// softmax(Q K^T / sqrt(64) [+ causal mask]) V for every (sequence, head), the SDPA that
// nn.MultiheadAttention dispatches in custom_clip_model.py:12,22-24 (vision: L = 211/213,
// no mask) and maple.py:956-962,976 (text: L = 77, additive -inf causal mask).
//
// One workgroup per (sequence, head), one wave per 32-query block.  K [Lp][64] and V^T
// [64][Lp] of the head live in LDS for the whole sweep (L <= 256 fits: one key sweep, no
// online rescaling).  Row max / row sum are in-lane plus one xor-shuffle (lane ^ 32).
// Inputs from the QKV GEMM epilogue: q,k [B*H][L][64] fp16, vt [B*H][64][Lp] fp16 (the
// reference's GPU dtype); P is rounded to fp16 for the P.V MFMAs.
// Output o [B*L][H*64] fp16 (token-major: the A operand of out_proj).
#include "common.h"

#include <type_traits>

namespace reidmi {

int attn_lpad(int L);

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

__device__ __forceinline__ int kswz(int r, int kc) { return r * 64 + ((kc ^ ((r >> 1) & 7)) << 3); }

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef float f32x2v __attribute__((ext_vector_type(2)));
typedef _Float16 f16x2v __attribute__((ext_vector_type(2)));

// fp32 -> fp16 (RNE) of a value that must be rounded to fp32 first: the opaque copy keeps the
// backend from merging the fma that produced x and this conversion into one v_fma_mixlo_f16
// (a single rounding to fp16, which differs from gemm.hip's in about 1 value in 1500)
__device__ __forceinline__ _Float16 f32_to_h(float x) {
    asm("" : "+v"(x));
    return (_Float16)x;
}

// one v_cvt_pk_f16_f32 (RNE) per pair, as gemm.hip's epilogues convert
__device__ __forceinline__ uint32_t cvt_pk_h(float a, float b) {
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2v{a, b}, f16x2v));
}

// fp16 pair (a * inv, b * inv), each product rounded to fp16 ONCE (v_fma_mixlo / mixhi: the
// exact product, one rounding).  Left to itself the backend lowers (_Float16)(a * inv) as a
// mix instruction for some elements and as v_mul + v_cvt_pk (two roundings) for others, so
// the two attention blocks would differ in ~1 value in 36 000.
__device__ __forceinline__ uint32_t mul_pk_h(float a, float b, float inv) {
#ifdef ATTN_OUT_CVT  // A/B only: fp32 product, then RNE to fp16 (two roundings)
    float x = a * inv, y = b * inv;
    asm("" : "+v"(x), "+v"(y));
    return cvt_pk_h(x, y);
#endif
    uint32_t r;
    asm("v_fma_mixlo_f16 %0, %1, %2, 0" : "=v"(r) : "v"(a), "v"(inv));
    asm("v_fma_mixhi_f16 %0, %1, %2, 0" : "+v"(r) : "v"(b), "v"(inv));
    return r;
}

// One wave's block of 32 queries (row qi = block * 32 + (lane & 31)) against the head's K
// [LP][64] and V^T [64][vstride] in LDS:
//   S^T[key][q] = K Q^T on v_mfma_f32_32x32x16_f16; lane (q = lane&31, h = lane>>5) holds
//     keys kb*32 + (r&3) + 8(r>>2) + 4h in s[kb][r];
//   P stays in registers: registers 8s'..8s'+7 of block kb are the B fragment of key-step s'
//     of O^T = V^T P^T (accumulator-as-operand), V^T read with the same key permutation;
//   O^T[d][q] comes out as 4 runs of 4 consecutive d per lane -> kAttnStores 8-byte stores (the
//     wave's only vector-memory ops here; lanes with qi >= L store nothing).
constexpr int kAttnStores = 8;  // (2 d blocks x 4 runs; the callers' counted waits use it)
template <int NKB, bool CAUSAL>
__device__ __forceinline__ void attn_block(const _Float16* sK, const _Float16* sV, int vstride, const f16x8 (&qf)[4],
                                           int qi, int L, int64_t bh, int H, _Float16* __restrict__ o,
                                           float scale_log2) {
    const int lane = threadIdx.x & 63;
    const int hh = lane >> 5, ql = lane & 31;
    f32x16 s[NKB];
#pragma unroll
    for (int kb = 0; kb < NKB; kb++) {
        f32x16 a = f32x16{};
#pragma unroll
        for (int ks = 0; ks < 4; ks++) {
            const f16x8 kf = *(const f16x8*)(sK + kswz(kb * 32 + ql, 2 * ks + hh));
            a = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf, qf[ks], a, 0, 0, 0);
        }
        s[kb] = a;
    }
    float mx = -__builtin_inff();
#pragma unroll
    for (int kb = 0; kb < NKB; kb++)
#pragma unroll
        for (int r = 0; r < 16; r++) {
            if (CAUSAL || kb == NKB - 1) {
                const int key = kb * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
                const bool ok = key < L && (!CAUSAL || key <= qi);
                s[kb][r] = ok ? s[kb][r] : -__builtin_inff();
            }
            mx = fmaxf(mx, s[kb][r]);
        }
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    // exponent argument and running sums on packed-fp32 VALU (v_pk_fma_f32 /
    // v_pk_add_f32: two elements per instruction); two partial sums (even / odd r).
    const float mb = -mx * scale_log2;
    const f32x2v sc2 = {scale_log2, scale_log2}, mb2 = {mb, mb};
    f32x2v sum2 = {0.f, 0.f};
#pragma unroll
    for (int kb = 0; kb < NKB; kb++)
#pragma unroll
        for (int r = 0; r < 16; r += 2) {
            const f32x2v t = __builtin_elementwise_fma(f32x2v{s[kb][r], s[kb][r + 1]}, sc2, mb2);
            const f32x2v p = {__builtin_amdgcn_exp2f(t.x), __builtin_amdgcn_exp2f(t.y)};
            s[kb][r] = p.x;
            s[kb][r + 1] = p.y;
            sum2 += p;
        }
    float sum = sum2.x + sum2.y;
    sum += __shfl_xor(sum, 32, 64);
    const float inv = 1.0f / sum;
    f32x16 oacc[2] = {f32x16{}, f32x16{}};
#pragma unroll
    for (int kb = 0; kb < NKB; kb++)
#pragma unroll
        for (int sp = 0; sp < 2; sp++) {
            f16x8 pf;
#pragma unroll
            for (int j = 0; j < 8; j++) pf[j] = (_Float16)s[kb][8 * sp + j];
#pragma unroll
            for (int db = 0; db < 2; db++) {
                const _Float16* vr = sV + (db * 32 + ql) * vstride + kb * 32 + 16 * sp + 4 * hh;
                const f16x4 v0 = *(const f16x4*)(vr);
                const f16x4 v1 = *(const f16x4*)(vr + 8);
                const f16x8 vf = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
                oacc[db] = __builtin_amdgcn_mfma_f32_32x32x16_f16(vf, pf, oacc[db], 0, 0, 0);
            }
        }
    if (qi < L) {
        const int64_t b = bh / H, hd = bh % H;
        _Float16* orow = o + (b * L + qi) * (int64_t)(H * 64) + hd * 64;
        static_assert(2 * 4 == kAttnStores, "one store per (d block, run)");
#pragma unroll
        for (int db = 0; db < 2; db++)
#pragma unroll
            for (int g = 0; g < 4; g++) {
                const uint2 w = make_uint2(mul_pk_h(oacc[db][4 * g], oacc[db][4 * g + 1], inv),
                                           mul_pk_h(oacc[db][4 * g + 2], oacc[db][4 * g + 3], inv));
                *(uint2*)(orow + db * 32 + 8 * g + 4 * hh) = w;
            }
    }
}

// ----------------------------------------------------------- software-pipelined block
// The same arithmetic as attn_block (bit-identical outputs: same MFMA chains, same max, same
// exp2 arguments, same order of the running sums, same RNE conversions), scheduled so that a
// wave never waits a whole LDS round trip in front of its MFMAs and its softmax VALU runs in
// the shadow of its own MFMAs:
//  * S phase: the K fragments of key block kb+1 are read (inline ds_read_b128, immediate
//    offsets) while the 4 MFMAs of block kb run; a counted lgkmcnt(4) retires only block kb's;
//    the max of block kb-1 is folded in beside block kb's MFMAs.
//  * P.V phase: V^T of block kb+1 is read (ds_read2_b64: v0 | v1 land as one f16x8 operand)
//    and the exp2 / sum / fp16 pack of block kb+1 are computed while block kb's MFMAs run.
//  * the cross-half exchanges (max, sum) use v_permlane32_swap: no LDS op of the compiler's
//    own in the block, so the counted waits are exact.
//  * O^T is widened to 16-byte stores by one v_permlane32_swap per dword (4 stores per lane
//    instead of 8 half-width ones): kAttnPipeStores vector-memory ops per wave.
constexpr int kAttnPipeStores = 4;
#ifndef ATTN_TEXT_STAGES  // LDS stages of the causal mhsa_kernel at NKB <= 4 (2: the plain double buffer)
#define ATTN_TEXT_STAGES 3
#endif
#ifndef ATTN_PIPE
#define ATTN_PIPE 1
#endif
#if !defined(REIDMI_TOOLS) && ATTN_PIPE != 1
#error "attention.hip: ATTN_PIPE variants build only with -DREIDMI_TOOLS (never into libreidmi.so)"
#endif

template <int I, int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        static_for<I + 1, N>(f);
    }
}

template <int OFF>
__device__ __forceinline__ void ds_rd128(f16x8& d, uint32_t a) {
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(d) : "v"(a), "n"(OFF) : "memory");
}
// two 8-byte reads 16 bytes apart (offsets in units of 8 bytes) -> one f16x8
template <int OFF8>
__device__ __forceinline__ void ds_rd2x64(f16x8& d, uint32_t a) {
    asm volatile("ds_read2_b64 %0, %1 offset0:%2 offset1:%3" : "=v"(d) : "v"(a), "n"(OFF8), "n"(OFF8 + 2) : "memory");
}
template <int N>
__device__ __forceinline__ void lgkm_wait4(f16x8& a, f16x8& b, f16x8& c, f16x8& d) {
    asm volatile("s_waitcnt lgkmcnt(%4)" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "n"(N) : "memory");
}
// {x[l], x[l ^ 32]} in some order per lane.  The results are copied out as uint32_t before any
// bit_cast: hipcc 7.2 lowers __builtin_bit_cast(float, r[1]) applied to the builtin's vector
// result as element 0 (both results then read the first register).
__device__ __forceinline__ void xhalf_pair(float x, float& a, float& b) {
    const uint32_t u = __builtin_bit_cast(uint32_t, x);
    const auto r = __builtin_amdgcn_permlane32_swap(u, u, false, false);
    const uint32_t r0 = r[0], r1 = r[1];
    a = __builtin_bit_cast(float, r0);
    b = __builtin_bit_cast(float, r1);
}
__device__ __forceinline__ float xhalf_max(float x) {  // max(x[l], x[l ^ 32])
    float a, b;
    xhalf_pair(x, a, b);
    return fmaxf(a, b);
}
__device__ __forceinline__ float xhalf_sum(float x) {  // x[l] + x[l ^ 32] (commutative: = x + shfl_xor(x, 32))
    float a, b;
    xhalf_pair(x, a, b);
    return a + b;
}

#ifdef ATTN_STAMPS
// diagnostic build only (tools/attn_stamps.py): s_memtime per phase of heads 8..15 of every
// workgroup, 8 stamps per (workgroup, wave, head)
__device__ uint64_t g_attn_stamps[256 * 8 * 8 * 8];
#define ATTN_STAMP(i) (stamp[i] = __builtin_amdgcn_s_memtime())
#else
#define ATTN_STAMP(i) ((void)0)
#endif

// mid(): called once in the P.V phase (after block NKB/2's MFMAs), after(): right after the
// last P.V MFMA, before the O stores — the caller's prefetch for the next head goes there.
template <int NKB, int VS_ = NKB * 32 + 4, typename Mid, typename After>
__device__ __forceinline__ void attn_block_pipe(const _Float16* sK, const _Float16* sV, const f16x8 (&qf)[4], int qi,
                                                int L, int64_t bh, int H, _Float16* __restrict__ o, float scale_log2,
                                                Mid&& mid, After&& after
#ifdef ATTN_STAMPS
                                                ,
                                                uint64_t* stamp
#endif
) {
    constexpr int VS = VS_;  // V^T row stride in LDS (mhsa_pipe_kernel: vt_stride(LP); mhsa_rr_kernel: 212)
    const int lane = threadIdx.x & 63;
    const int hh = lane >> 5, ql = lane & 31;
    // K fragment bases (one per 16-wide k-step; the key block is an immediate: the swizzle
    // term depends on the row only through (row >> 1) & 7 = (ql >> 1) & 7)
    uint32_t ka[4];
#pragma unroll
    for (int ks = 0; ks < 4; ks++) ka[ks] = lds_addr(sK + ql * 64 + (((2 * ks + hh) ^ ((ql >> 1) & 7)) << 3));
    // V^T bases of the two 32-row d blocks; key block / half-step offsets are immediates
    const uint32_t va0 = lds_addr(sV + ql * VS + 4 * hh), va1 = va0 + 32 * VS * 2;

    f32x16 s[NKB];
    f16x8 kf[2][4];
    float mx = -__builtin_inff();
    auto rd_k = [&](auto kbc) {
        constexpr int kb = decltype(kbc)::value;
        ds_rd128<kb * 32 * 64 * 2>(kf[kb & 1][0], ka[0]);
        ds_rd128<kb * 32 * 64 * 2>(kf[kb & 1][1], ka[1]);
        ds_rd128<kb * 32 * 64 * 2>(kf[kb & 1][2], ka[2]);
        ds_rd128<kb * 32 * 64 * 2>(kf[kb & 1][3], ka[3]);
    };
    auto fold_max = [&](auto kbc) {
        constexpr int kb = decltype(kbc)::value;
        if constexpr (kb == NKB - 1) {
#pragma unroll
            for (int r = 0; r < 16; r++) {
                const int key = kb * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
                s[kb][r] = key < L ? s[kb][r] : -__builtin_inff();
            }
        }
        // two independent chains (max is exact: any order gives the same value), pinned into
        // this block's slot (a volatile asm keeps its place among the reads / waits)
        float m0 = s[kb][0], m1 = s[kb][1];
#pragma unroll
        for (int r = 2; r < 16; r += 4) {
            m0 = fmaxf(m0, fmaxf(s[kb][r], s[kb][r + 1]));
            m1 = fmaxf(m1, fmaxf(s[kb][r + 2], s[kb][r + 3]));
        }
        mx = fmaxf(mx, fmaxf(m0, m1));
        asm volatile("" : "+v"(mx));
    };
    rd_k(std::integral_constant<int, 0>{});
    static_for<0, NKB>([&](auto kbc) {
        constexpr int kb = decltype(kbc)::value;
        if constexpr (kb + 1 < NKB) {
            rd_k(std::integral_constant<int, kb + 1>{});
            lgkm_wait4<4>(kf[kb & 1][0], kf[kb & 1][1], kf[kb & 1][2], kf[kb & 1][3]);
        } else {
            lgkm_wait4<0>(kf[kb & 1][0], kf[kb & 1][1], kf[kb & 1][2], kf[kb & 1][3]);
        }
        f32x16 a = f32x16{};
#pragma unroll
        for (int ks = 0; ks < 4; ks++) a = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf[kb & 1][ks], qf[ks], a, 0, 0, 0);
        s[kb] = a;
        if constexpr (kb > 0) fold_max(std::integral_constant<int, kb - 1>{});
    });
    fold_max(std::integral_constant<int, NKB - 1>{});
    mx = xhalf_max(mx);
    ATTN_STAMP(2);

    const float mb = -mx * scale_log2;
    const f32x2v sc2 = {scale_log2, scale_log2}, mb2 = {mb, mb};
    f32x2v sum2 = {0.f, 0.f};
    f16x8 vf[2][2][2];  // [kb parity][sp][db]
    f16x8 pf[2][2];     // [kb parity][sp]
    auto rd_v = [&](auto kbc) {
        constexpr int kb = decltype(kbc)::value;
        ds_rd2x64<(kb * 64 + 0) / 8>(vf[kb & 1][0][0], va0);
        ds_rd2x64<(kb * 64 + 0) / 8>(vf[kb & 1][0][1], va1);
        ds_rd2x64<(kb * 64 + 32) / 8>(vf[kb & 1][1][0], va0);
        ds_rd2x64<(kb * 64 + 32) / 8>(vf[kb & 1][1][1], va1);
    };
    auto softmax_blk = [&](auto kbc) {  // exp2 + running sums + fp16 pack of key block kb
        constexpr int kb = decltype(kbc)::value;
#pragma unroll
        for (int r = 0; r < 16; r += 2) {
            const f32x2v t = __builtin_elementwise_fma(f32x2v{s[kb][r], s[kb][r + 1]}, sc2, mb2);
            const f32x2v p = {__builtin_amdgcn_exp2f(t.x), __builtin_amdgcn_exp2f(t.y)};
            s[kb][r] = p.x;
            s[kb][r + 1] = p.y;
            sum2 += p;
        }
        // the running sums stay in this block's slot (left alone, the compiler sinks all 56
        // dependent adds to the end of the phase: a serial chain behind the last MFMA)
        asm volatile("" : "+v"(sum2));
#pragma unroll
        for (int sp = 0; sp < 2; sp++)
#pragma unroll
            for (int j = 0; j < 8; j++) pf[kb & 1][sp][j] = (_Float16)s[kb][8 * sp + j];
    };
    f32x16 oacc[2] = {f32x16{}, f32x16{}};
    rd_v(std::integral_constant<int, 0>{});
    softmax_blk(std::integral_constant<int, 0>{});
    static_for<0, NKB>([&](auto kbc) {
        constexpr int kb = decltype(kbc)::value;
        if constexpr (kb + 1 < NKB) {
            rd_v(std::integral_constant<int, kb + 1>{});
            lgkm_wait4<4>(vf[kb & 1][0][0], vf[kb & 1][0][1], vf[kb & 1][1][0], vf[kb & 1][1][1]);
        } else {
            lgkm_wait4<0>(vf[kb & 1][0][0], vf[kb & 1][0][1], vf[kb & 1][1][0], vf[kb & 1][1][1]);
            // V^T key columns >= L hold whatever the DMA brought (the HBM row padding): zero
            // them in registers (P is exactly 0 there; 0 * NaN would not be), so no pass over
            // the LDS pad is needed.  Half e of a fragment is key kb*32 + 16 sp + 4 hh + (e & 3)
            // + 8 (e >> 2); dword j holds halves 2j, 2j + 1.
#pragma unroll
            for (int sp = 0; sp < 2; sp++) {
                uint32_t m[4];
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const int key = kb * 32 + 16 * sp + 4 * hh + (2 * j & 3) + 8 * (j >> 1);
                    m[j] = key >= L ? 0u : key + 1 >= L ? 0x0000ffffu : 0xffffffffu;
                }
#pragma unroll
                for (int db = 0; db < 2; db++) {
                    uint4 u = __builtin_bit_cast(uint4, vf[kb & 1][sp][db]);
                    u.x &= m[0];
                    u.y &= m[1];
                    u.z &= m[2];
                    u.w &= m[3];
                    vf[kb & 1][sp][db] = __builtin_bit_cast(f16x8, u);
                }
            }
        }
#pragma unroll
        for (int sp = 0; sp < 2; sp++)
#pragma unroll
            for (int db = 0; db < 2; db++)
                oacc[db] = __builtin_amdgcn_mfma_f32_32x32x16_f16(vf[kb & 1][sp][db], pf[kb & 1][sp], oacc[db], 0, 0, 0);
        if constexpr (kb + 1 < NKB) softmax_blk(std::integral_constant<int, kb + 1>{});
        if constexpr (kb == NKB / 2) mid();
    });
    after();
    const float sum = xhalf_sum(sum2.x + sum2.y);
    const float inv = 1.0f / sum;
    ATTN_STAMP(3);
    // lane (ql, hh) holds d = db*32 + 8g + 4hh + 0..3; pair g = 2j, 2j+1 across the halves so
    // that half 0 stores d 16j..16j+7 and half 1 d 16j+8..16j+15 (16 bytes each)
    uint4 w[2][2];
#pragma unroll
    for (int db = 0; db < 2; db++)
#pragma unroll
        for (int j = 0; j < 2; j++) {
            const int g0 = 2 * j, g1 = 2 * j + 1;
            auto pk = [&](int e) { return mul_pk_h(oacc[db][e], oacc[db][e + 1], inv); };
            const uint32_t x0 = pk(4 * g0), x1 = pk(4 * g0 + 2), y0 = pk(4 * g1), y1 = pk(4 * g1 + 2);
            const auto r0 = __builtin_amdgcn_permlane32_swap(x0, y0, false, false);
            const auto r1 = __builtin_amdgcn_permlane32_swap(x1, y1, false, false);
            w[db][j] = make_uint4(r0[0], r1[0], r0[1], r1[1]);
        }
    if (qi < L) {
        const int64_t b = bh / H, hd = bh % H;
        _Float16* orow = o + (b * L + qi) * (int64_t)(H * 64) + hd * 64 + 8 * hh;
#pragma unroll
        for (int db = 0; db < 2; db++)
#pragma unroll
            for (int j = 0; j < 2; j++) *(uint4*)(orow + db * 32 + 16 * j) = w[db][j];
    }
}

// Persistent: gridDim.x workgroups (one per CU) walk the (sequence, head) pairs; one wave
// per 32-query block (ceil(L/32) waves).  NKB = number of 32-key blocks (Lp = 32 * NKB).
// K of the next head is copied into the other LDS stage by global_load_lds (8 rows per 1-KiB
// piece, XOR swizzle applied on the source address) and V^T of the next head as one
// contiguous blob (its HBM row stride == its LDS row stride, see attn_lpad), both while
// the current head is being computed; Q of the next head is prefetched into registers.
//   S^T[key][q] = K Q^T on v_mfma_f32_32x32x16_f16; lane (q = lane&31, h = lane>>5) holds
//     keys kb*32 + (r&3) + 8(r>>2) + 4h in s[kb][r];
//   P stays in registers: registers 8s'..8s'+7 of block kb are the B fragment of key-step s'
//     of O^T = V^T P^T (accumulator-as-operand), V^T read with the same key permutation;
//   O^T[d][q] comes out as 4 runs of 4 consecutive d per lane -> 8-byte stores.

//   NS = 3 (the causal text shapes, NKB <= 4): a ring of three LDS stages, K/V two heads ahead
//   and Q one head ahead — short text heads are bound by the latency of their loads (one head
//   in flight per workgroup left the CU waiting).
template <int NKB, bool CAUSAL, int NS = 2>
__global__ __launch_bounds__(512) void mhsa_kernel(const _Float16* __restrict__ q, const _Float16* __restrict__ k,
                                                   const _Float16* __restrict__ vt, _Float16* __restrict__ o, int L,
                                                   int H, int vstride, int64_t nbh, float scale_log2) {
    constexpr int LP = NKB * 32;
    extern __shared__ __attribute__((aligned(16))) _Float16 lds[];
    const int stage_elems = LP * 64 + 64 * vstride;  // K [LP][64] then V^T [64][vstride]
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int nw = blockDim.x >> 6;
    const int hh = lane >> 5, ql = lane & 31;
    const int qi = wid * 32 + ql;
    const int kpieces = LP / 8;                           // 1-KiB pieces of K
    const int vbytes = 64 * vstride * 2;                   // V^T blob (a multiple of 512 B)
    const int vpieces = (vbytes + 1023) / 1024;             // 1-KiB pieces; last may be half
    const int vlast_lanes = (vbytes - (vpieces - 1) * 1024) / 16;

    auto issue = [&](int64_t bh, int stage) {
        _Float16* sK = lds + stage * stage_elems;
        _Float16* sV = sK + LP * 64;
        const _Float16* kh = k + bh * L * 64;
        const _Float16* vh = vt + bh * 64 * (int64_t)vstride;
        for (int pc = wid; pc < kpieces; pc += nw) {
            int r = 8 * pc + (lane >> 3);
            const int kc = (lane & 7) ^ ((r >> 1) & 7);
            r = r < L ? r : L - 1;  // rows >= L: any finite key (masked to -inf below)
            __builtin_amdgcn_global_load_lds(kh + (int64_t)r * 64 + kc * 8, (lds_ptr_t)(sK + pc * 512), 16, 0, 0);
        }
        for (int pc = wid; pc < vpieces; pc += nw)
            if (pc + 1 < vpieces || lane < vlast_lanes)  // never read or write past the blob
                __builtin_amdgcn_global_load_lds(vh + pc * 512 + lane * 8, (lds_ptr_t)(sV + pc * 512), 16, 0, 0);
    };
    // Q rows of this wave's queries; queries >= L load row L-1 (finite; never stored).
    // Inline-asm loads: hipcc does not track them, so it inserts no vmcnt(0) of its own
    // before the prefetched registers are used (which would also drain the O stores); the
    // kernel's counted waits retire them, and `pin` orders every use after that wait.
    auto load_q = [&](int64_t bh, f16x8* qf) {
        const _Float16* qh = q + (bh * L + (qi < L ? qi : L - 1)) * 64 + hh * 8;
        asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(qf[0]) : "v"(qh) : "memory");
        asm volatile("global_load_dwordx4 %0, %1, off offset:32" : "=v"(qf[1]) : "v"(qh) : "memory");
        asm volatile("global_load_dwordx4 %0, %1, off offset:64" : "=v"(qf[2]) : "v"(qh) : "memory");
        asm volatile("global_load_dwordx4 %0, %1, off offset:96" : "=v"(qf[3]) : "v"(qh) : "memory");
    };
    auto pin = [&](f16x8* qf) {
        asm volatile("" : "+v"(qf[0]), "+v"(qf[1]), "+v"(qf[2]), "+v"(qf[3]));
    };
    auto zero_pad = [&](int stage) {  // V^T key columns [L, LP) were DMA'd from padding
        _Float16* sV = lds + stage * stage_elems + LP * 64;
        for (int c = tid; c < 64 * (LP - L); c += blockDim.x) {
            const int d = c / (LP - L), t = L + c % (LP - L);
            sV[d * vstride + t] = (_Float16)0.0f;
        }
    };

    int64_t bh = blockIdx.x;
    if (bh >= nbh) return;
    if constexpr (NS == 3) {
        // The counted waits below are derived from the per-wave vector-memory ops of a head
        // (ADVICE r4): with nw == NKB waves and V^T rows of LP + 4 (both checked by the
        // launcher) every wave issues kRingK K pieces and kRingV V^T pieces per head, wave 0 one
        // more (the blob's half last piece); attn_block issues kAttnStores O stores and load_q 4
        // loads.  Each is one instruction (1-KiB LDS-DMA pieces, 8-byte stores: nothing to merge
        // or split), and the kernels use no scratch (tests/test_capi.py checks the ISA).
        constexpr int kRingK = LP / 8 / NKB, kRingV = 4;
        static_assert(kRingK == 4, "K: 4 one-KiB pieces per wave and head");
        static_assert((64 * (LP + 4) * 2 + 1023) / 1024 == kRingV * NKB + 1, "V^T: 4 pieces per wave + wave 0's half");
        constexpr int kIssue = kRingK + kRingV;        // one head's K / V^T pieces, waves 1..
        constexpr int kIssue0 = kIssue + 1;            // wave 0
        const int64_t G = gridDim.x;
        issue(bh, 0);
        f16x8 qf[4];
        load_q(bh, qf);
        const bool second = bh + G < nbh;
        if (second) issue(bh + G, 1);
        // the first head's K / V^T and Q have landed; the second head's K / V^T stays in flight
        if (!second)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        else if (wid == 0)
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kIssue0) : "memory");
        else
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kIssue) : "memory");
        pin(qf);
        __builtin_amdgcn_s_barrier();
        zero_pad(0);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        int stage = 0;
        for (; bh < nbh; bh += G) {
            const int64_t nxt = bh + G, nxt2 = bh + 2 * G;
            f16x8 qn[4];
            if (nxt < nbh) load_q(nxt, qn);  // issued before the K/V of nxt2: retired with nxt's
            if (nxt2 < nbh) issue(nxt2, stage == 0 ? 2 : stage - 1);  // the stage head bh-G used
            const _Float16* sK = lds + stage * stage_elems;
            const _Float16* sV = sK + LP * 64;
            if (wid * 32 < L) attn_block<NKB, CAUSAL>(sK, sV, vstride, qf, qi, L, bh, H, o, scale_log2);
            // nxt's K / V^T (issued one head ago) and Q have landed; nxt2's K / V^T and this
            // head's O stores (the youngest ops) stay in flight
            if (wid * 32 >= L)
                asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
            else if (nxt2 >= nbh)
                asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(kAttnStores) : "memory");
            else if (wid == 0)
                asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(kIssue0 + kAttnStores) : "memory");
            else
                asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(kIssue + kAttnStores) : "memory");
            __builtin_amdgcn_s_barrier();
            const int nstage = stage == 2 ? 0 : stage + 1;
            if (nxt < nbh) {
                zero_pad(nstage);
                pin(qn);
#pragma unroll
                for (int ks = 0; ks < 4; ks++) qf[ks] = qn[ks];
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            stage = nstage;
        }
        return;
    }
    int stage = 0;
    issue(bh, 0);
    f16x8 qf[4];
    load_q(bh, qf);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    pin(qf);
    __syncthreads();
    zero_pad(0);
    __syncthreads();
    for (; bh < nbh; bh += gridDim.x) {
        const int64_t nxt = bh + gridDim.x;
        f16x8 qn[4];
        if (nxt < nbh) {  // Q first: the compiler's wait for qn then never covers the DMA
            load_q(nxt, qn);
            issue(nxt, stage ^ 1);
        }
        const _Float16* sK = lds + stage * stage_elems;
        const _Float16* sV = sK + LP * 64;
        if (wid * 32 < L) attn_block<NKB, CAUSAL>(sK, sV, vstride, qf, qi, L, bh, H, o, scale_log2);
        // Wait for the next head's K/V DMA and Q loads only: the 8 O stores this wave just
        // issued (when it owns queries) are the youngest vector-memory ops and stay in flight
        // (vmcnt retires in issue order).
        // Raw barriers: __syncthreads() would add a vmcnt(0) (a workgroup release covers the
        // stores) and drain them anyway.  LDS-DMA data is ordered for other waves' ds_reads
        // by each issuing wave's vmcnt + this barrier; zero_pad's ds_writes by lgkmcnt(0).
        if (wid * 32 < L)
            asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(kAttnStores) : "memory");
        else
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (nxt < nbh) {
            zero_pad(stage ^ 1);
            pin(qn);
#pragma unroll
            for (int ks = 0; ks < 4; ks++) qf[ks] = qn[ks];
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        stage ^= 1;
    }
}

// Non-causal blocks (the vision towers): the software-pipelined attn_block_pipe, with the
// next head's prefetch split by wave age.  Waves w and w + 4 share a SIMD; the younger one
// (w >= 4) loses every MFMA / VALU arbitration to the older, so it runs the critical path
// (phase stamps, tools/attn_stamps.py: before this split the younger waves' S phase took 2.2x
// the older ones', and the older waves then idled ~3k cycles per head at the barrier):
//  * waves 0-3 issue the next head's K (LDS-DMA) and their own next Q rows at the head start,
//    and the next head's V^T blob right after their last P.V MFMA (V is needed only by the
//    next head's P.V phase: most of a head of lead time; those waves idled ~3-4k cycles per
//    head at the barrier);
//  * waves 4.. only load their own next Q rows, in the middle of their P.V phase;
//  * the V^T key padding is zeroed in registers (attn_block_pipe), so a head needs one
//    barrier: each wave waits for its own prefetch (its O stores stay in flight), barrier.
template <int NKB>
__global__ __launch_bounds__(NKB * 64) void mhsa_pipe_kernel(const _Float16* __restrict__ q,
                                                            const _Float16* __restrict__ k,
                                                            const _Float16* __restrict__ vt, _Float16* __restrict__ o,
                                                            int L, int H, int64_t nbh, float scale_log2) {
    constexpr int LP = NKB * 32, VS = LP + 4, NW = NKB;
    constexpr int NOLD = NW > 4 ? 4 : NW;              // waves issuing K (and V when NW <= 4)
    constexpr int STAGE = LP * 64 + 64 * VS;           // K [LP][64] then V^T [64][VS]
    constexpr int KPIECES = LP / 8;                    // 1-KiB pieces of K
    constexpr int VBYTES = 64 * VS * 2;                // V^T blob (a multiple of 512 B)
    constexpr int VPIECES = (VBYTES + 1023) / 1024;    // last may be half
    constexpr int VLAST = (VBYTES - (VPIECES - 1) * 1024) / 16;
    extern __shared__ __attribute__((aligned(16))) _Float16 lds[];
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int hh = lane >> 5, ql = lane & 31;
    const int qi = wid * 32 + ql;

    auto issue_k = [&](int64_t bh, int stage, int w0, int nws) {
        _Float16* sK = lds + stage * STAGE;
        const _Float16* kh = k + bh * L * 64;
        for (int pc = wid - w0; pc < KPIECES; pc += nws) {
            int r = 8 * pc + (lane >> 3);
            const int kc = (lane & 7) ^ ((r >> 1) & 7);
            r = r < L ? r : L - 1;  // rows >= L: any finite key (masked to -inf)
            __builtin_amdgcn_global_load_lds(kh + (int64_t)r * 64 + kc * 8, (lds_ptr_t)(sK + pc * 512), 16, 0, 0);
        }
    };
    auto issue_v = [&](int64_t bh, int stage, int w0, int nws) {
        _Float16* sV = lds + stage * STAGE + LP * 64;
        const _Float16* vh = vt + bh * 64 * (int64_t)VS;
        for (int pc = wid - w0; pc < VPIECES; pc += nws)
            if (pc + 1 < VPIECES || lane < VLAST)  // never read or write past the blob
                __builtin_amdgcn_global_load_lds(vh + pc * 512 + lane * 8, (lds_ptr_t)(sV + pc * 512), 16, 0, 0);
    };
    // Q rows of this wave's queries (rows >= L read row L-1: finite, never stored); inline-asm
    // loads, retired by the kernel's counted waits, every use ordered after them by pin()
    auto load_q = [&](int64_t bh, f16x8* qf) {
        const _Float16* qh = q + (bh * L + (qi < L ? qi : L - 1)) * 64 + hh * 8;
        asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(qf[0]) : "v"(qh) : "memory");
        asm volatile("global_load_dwordx4 %0, %1, off offset:32" : "=v"(qf[1]) : "v"(qh) : "memory");
        asm volatile("global_load_dwordx4 %0, %1, off offset:64" : "=v"(qf[2]) : "v"(qh) : "memory");
        asm volatile("global_load_dwordx4 %0, %1, off offset:96" : "=v"(qf[3]) : "v"(qh) : "memory");
    };
    auto pin = [&](f16x8* qf) { asm volatile("" : "+v"(qf[0]), "+v"(qf[1]), "+v"(qf[2]), "+v"(qf[3])); };

    int64_t bh = blockIdx.x;
    if (bh >= nbh) return;
    int stage = 0;
    issue_k(bh, 0, 0, NW);
    issue_v(bh, 0, 0, NW);
    f16x8 qf[4];
    load_q(bh, qf);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    pin(qf);
    __builtin_amdgcn_s_barrier();
#ifdef ATTN_STAMPS
    uint64_t stamp[8] = {};
    int it = 0;
#endif
    for (; bh < nbh; bh += gridDim.x) {
        ATTN_STAMP(0);
        const int64_t nxt = bh + gridDim.x;
        const bool more = nxt < nbh;
        f16x8 qn[4];
        if (more && wid < NOLD) {
            load_q(nxt, qn);
            issue_k(nxt, stage ^ 1, 0, NOLD);
        }
        ATTN_STAMP(1);
        const _Float16* sK = lds + stage * STAGE;
        attn_block_pipe<NKB>(
            sK, sK + LP * 64, qf, qi, L, bh, H, o, scale_log2,
            [&] {
                if (more && wid >= NOLD) load_q(nxt, qn);
            },
            [&] {
                if (more && wid < NOLD) issue_v(nxt, stage ^ 1, 0, NOLD);
            }
#ifdef ATTN_STAMPS
            ,
            stamp
#endif
        );
        // this wave's prefetch has landed; its kAttnPipeStores O stores (the youngest
        // vector-memory ops) stay in flight.  A raw barrier (__syncthreads would drain them).
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kAttnPipeStores) : "memory");
        ATTN_STAMP(4);
        __builtin_amdgcn_s_barrier();
        ATTN_STAMP(5);
        if (more) {
            pin(qn);
#pragma unroll
            for (int ks = 0; ks < 4; ks++) qf[ks] = qn[ks];
        }
        stage ^= 1;
#ifdef ATTN_STAMPS
        if (it >= 8 && it < 16 && lane == 0 && blockIdx.x < 256) {
            uint64_t* d = g_attn_stamps + ((blockIdx.x * 8 + wid) * 8 + (it - 8)) * 8;
            for (int i = 0; i < 6; i++) d[i] = stamp[i];
        }
        it++;
#endif
    }
}

// ----------------------------------------------------------- round-robin units (round 6)
// Built only into the tools library (libreidmi_tools.so, REIDMI_TOOLS): bit-exact with
// mhsa_pipe_kernel and measured no faster (profiles/r06/attn_rr_ab.txt), so the
// product library does not ship it.
// mhsa_pipe_kernel runs one (sequence, head) at a time on ceil(L/32) = 7 waves, and 7 waves on
// a CU's 4 SIMDs leave three SIMDs with two waves and one with one: a head's time follows the
// busiest SIMD (2 units of 32 queries), 8/7 of the balanced 7/4 (the round-5
// length scan).  Here 8 waves walk the workgroup's (head, 32-query block) UNITS round-robin:
// round r gives wave w unit u = 8r + w of the workgroup's sequence (local head j = u / NKB,
// block u % NKB; global head blockIdx.x + j * gridDim.x), so every SIMD runs two units per
// round and a round completes 8/7 heads.  A round touches at most two heads; three LDS slots
// hold them and the head the next round adds, slot j % 3 — K [VS][64] (rows < L written,
// XOR-swizzled as in mhsa_pipe_kernel) + V^T [64][VS] with VS = 212 for L in 205..212 (the
// caller's V^T rows; 212 = 4 mod 8 keeps the P.V reads conflict-free): 3 x 54 272 B + 64 B of read
// overhang = 162 880 B.  The reads past a slot's K rows or V^T columns are the masked keys of
// attn_block_pipe (scores replaced by -inf, V^T zeroed in registers), as in mhsa_pipe_kernel.
// Loads of the head the next round adds (wave-uniform schedule): its slot's previous head either
// finished before this round — the older waves issue its K at the round's start and its V^T after
// their P.V (as mhsa_pipe_kernel's prefetch) — or its last unit is this round's unit 8r (wave 0's;
// once every 7 rounds, when the next round adds two heads): wave 0 then issues the new head's K
// after its own S phase (mid) and its V^T after its own P.V (after), so the slot is refilled
// right behind its last reader.  One barrier per round; each wave's own loads are retired by
// vmcnt(kAttnPipeStores) in front of it (its O stores stay in flight).  Same arithmetic as
// mhsa_pipe_kernel (attn_block_pipe): bit-identical outputs.
#ifdef REIDMI_TOOLS
constexpr int kRrWaves = 8, kRrSlots = 3;
constexpr int kRrVS = 212, kRrLmin = 205;  // V^T rows of kRrVS for L in [kRrLmin, kRrVS]

template <int NKB, int VS>
__global__ __launch_bounds__(kRrWaves * 64, 1) void mhsa_rr_kernel(const _Float16* __restrict__ q,
                                                                 const _Float16* __restrict__ k,
                                                                 const _Float16* __restrict__ vt,
                                                                 _Float16* __restrict__ o, int L, int H,
                                                                 int64_t nbh, float scale_log2) {
    constexpr int NW = kRrWaves, NS = kRrSlots;
    constexpr int KR = VS;                              // K rows per slot (>= L)
    constexpr int SLOT = KR * 64 + 64 * VS;             // halves
    constexpr int KPIECES = (KR + 7) / 8;               // 1-KiB pieces of 8 K rows (rows >= L skipped)
    constexpr int VBYTES = 64 * VS * 2;                 // V^T blob: its HBM row stride == VS
    constexpr int VPIECES = (VBYTES + 1023) / 1024;     // the last may be partial
    constexpr int VLAST = (VBYTES - (VPIECES - 1) * 1024) / 16;
    static_assert(VS % 8 == 4 && VBYTES % 16 == 0, "V^T row stride: 2 mod 4 dwords");
    static_assert(NKB >= 7, "8 consecutive units must span at most two heads (three slots)");
    extern __shared__ __attribute__((aligned(16))) _Float16 lds[];
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int hh = lane >> 5, ql = lane & 31;
    const int G = (int)gridDim.x, b0 = (int)blockIdx.x;
    // this workgroup's heads j = 0 .. nh-1 are the global heads b0 + j * G (nbh < 2^31: the caller)
    const int nh = (int)((nbh - b0 + G - 1) / G);
    if (nh <= 0) return;
    const int U = nh * NKB, R = (U + NW - 1) / NW;
    auto head_k = [&](int j) { return k + ((int64_t)b0 + (int64_t)j * G) * L * 64; };
    auto head_v = [&](int j) { return vt + ((int64_t)b0 + (int64_t)j * G) * 64 * VS; };
    auto slot = [&](int j) { return lds + (j % NS) * SLOT; };

    auto issue_k = [&](const _Float16* kh, _Float16* sK, int first, int step) {
#pragma unroll 1
        for (int pc = first; pc < KPIECES; pc += step) {
            const int r = 8 * pc + (lane >> 3);
            const int kc = (lane & 7) ^ ((r >> 1) & 7);
            if (r < L)
                __builtin_amdgcn_global_load_lds(kh + r * 64 + kc * 8, (lds_ptr_t)(sK + pc * 512), 16, 0, 0);
        }
    };
    auto issue_v = [&](const _Float16* vh, _Float16* sV, int first, int step) {
#pragma unroll 1
        for (int pc = first; pc < VPIECES; pc += step)
            if (pc + 1 < VPIECES || lane < VLAST)  // never read or write past the blob
                __builtin_amdgcn_global_load_lds(vh + pc * 512 + lane * 8, (lds_ptr_t)(sV + pc * 512), 16, 0, 0);
    };
    // Q rows of unit u's queries (rows >= L read row L-1: finite, never stored); inline-asm
    // loads retired by the round's counted wait, every use ordered after it by pin()
    auto q_row = [&](int u) {
        const int j = u / NKB;
        const int qi = (u - j * NKB) * 32 + ql;
        return q + (((int64_t)b0 + (int64_t)j * G) * L + (qi < L ? qi : L - 1)) * 64 + hh * 8;
    };
    auto load_q = [&](const _Float16* qh, f16x8* qf) {
        asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(qf[0]) : "v"(qh) : "memory");
        asm volatile("global_load_dwordx4 %0, %1, off offset:32" : "=v"(qf[1]) : "v"(qh) : "memory");
        asm volatile("global_load_dwordx4 %0, %1, off offset:64" : "=v"(qf[2]) : "v"(qh) : "memory");
        asm volatile("global_load_dwordx4 %0, %1, off offset:96" : "=v"(qf[3]) : "v"(qh) : "memory");
    };
    auto pin = [&](f16x8* qf) { asm volatile("" : "+v"(qf[0]), "+v"(qf[1]), "+v"(qf[2]), "+v"(qf[3])); };

    // prologue: the heads of round 0, and each wave's first Q
    int loaded = (NW - 1) / NKB < nh - 1 ? (NW - 1) / NKB : nh - 1;  // last head whose loads are issued
    for (int j = 0; j <= loaded; j++) {
        issue_k(head_k(j), slot(j), wid, NW);
        issue_v(head_v(j), slot(j) + KR * 64, wid, NW);
    }
    f16x8 qf[4];
    if (wid < U) load_q(q_row(wid), qf);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    pin(qf);
    __builtin_amdgcn_s_barrier();
    const bool older = wid < 4;
    for (int r = 0; r < R; r++) {
        const int u = r * NW + wid, un = u + NW;
        // this round's heads: issued in earlier rounds by the schedule below; one it cannot cover
        // is loaded here with everyone waiting (never taken for NKB = 7 and 8 waves: kept so any
        // shape stays correct)
        {
            const int need = (r * NW + NW - 1 < U ? r * NW + NW - 1 : U - 1) / NKB;
            if (loaded < need) {
                for (int j = loaded + 1; j <= need; j++) {
                    issue_k(head_k(j), slot(j), wid, NW);
                    issue_v(head_v(j), slot(j) + KR * 64, wid, NW);
                }
                loaded = need;
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __builtin_amdgcn_s_barrier();
            }
        }
        // the head(s) the next round adds: pa (its slot's head finished before this round) and
        // pb (its slot's head ends with this round's unit r * NW, wave 0's); wave-uniform
        int pa = -1, pb = -1;
        if ((r + 1) * NW < U) {
            const int need = ((r + 1) * NW + NW - 1 < U ? (r + 1) * NW + NW - 1 : U - 1) / NKB;
            while (loaded < need) {
                const int c = loaded + 1, prev_end = (c - NS) * NKB + NKB - 1;
                if ((c < NS || prev_end < r * NW) && pa < 0) {
                    pa = c;
                } else if (prev_end == r * NW && pb < 0) {
                    pb = c;
                } else {
                    break;
                }
                loaded = c;
            }
        }
        // pa's loads are shared by the older waves (waves 1-3 when wave 0 carries pb's)
        const int w0 = pb >= 0 ? 1 : 0, nws = 4 - w0;
        const bool share_a = pa >= 0 && older && wid >= w0;
        const bool carry_b = pb >= 0 && wid == 0;
        const _Float16* ka = share_a ? head_k(pa) : k;
        const _Float16* va = share_a ? head_v(pa) : vt;
        _Float16* sa = slot(share_a ? pa : 0);
        const _Float16* kb = carry_b ? head_k(pb) : k;
        const _Float16* vb = carry_b ? head_v(pb) : vt;
        _Float16* sb = slot(carry_b ? pb : 0);
        const _Float16* qn_row = q_row(un < U ? un : 0);
        f16x8 qn[4];
        if (share_a) issue_k(ka, sa, wid - w0, nws);
        if (un < U && older) load_q(qn_row, qn);
        if (u < U) {
            const int j = u / NKB;
            const _Float16* sK = slot(j);
            attn_block_pipe<NKB, VS>(
                sK, sK + KR * 64, qf, (u - j * NKB) * 32 + ql, L, (int64_t)b0 + (int64_t)j * G, H, o, scale_log2,
                [&] {
                    if (un < U && !older) load_q(qn_row, qn);
                    if (carry_b) issue_k(kb, sb, 0, 1);  // after this wave's S phase: its K is no longer read
                },
                [&] {
                    if (share_a) issue_v(va, sa + KR * 64, wid - w0, nws);
                    if (carry_b) issue_v(vb, sb + KR * 64, 0, 1);  // after its P.V: its V^T is no longer read
                });
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kAttnPipeStores) : "memory");
        } else {  // no unit this round (the last round only; no next-round loads then)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __builtin_amdgcn_s_barrier();
        if (un < U) {
            pin(qn);
#pragma unroll
            for (int ks = 0; ks < 4; ks++) qf[ks] = qn[ks];
        }
    }
}
#endif  // REIDMI_TOOLS (round-robin vision attention)

// ======================================================== fused QKV GEMM + attention
// Built only into the tools library (libreidmi_tools.so, REIDMI_TOOLS): bit-exact with the
// two-kernel block and measured slower, so the product library does not ship it.
#ifdef REIDMI_TOOLS
// ln_1 -> in_proj -> SDPA of a vision block (custom_clip_model.py:12,22-27) in one persistent
// kernel: the QKV GEMM's 1 GB of q / k / v^T per batch of 1024 crops (and the attention's read
// of it) never reaches HBM.  Unit = (image b, head h): the 192 columns [q_h | k_h | v_h] of the
// LayerNorm-folded QKV GEMM over the image's NKB*32 (padded) token rows, K = width in steps of
// 32, then attention of the head from LDS.  One wave per 32 token rows (= its 32 queries).
//  * GEMM: exactly the MFMA chain of gemm.hip (v_mfma_f32_16x16x32_f16, W fragment as A, the
//    same 8-halves-per-lane k assignment, K ascending) and the same fold / bias epilogue and
//    RNE conversions, so q / k / v are bit-identical to gemm_f16(EPI_QKV) and the attention
//    (attn_block, the same code as mhsa_kernel) sees the same operands: the fused block equals
//    the unfused one bit for bit (tests/test_gpu_encoder.py test_qkv_attention_fused_bitexact).
//  * operands HBM/L2 -> LDS by global_load_lds (1 KiB pieces: 16 rows x 64 B), a 3-stage ring
//    of K-steps that runs on across units (the next unit's first two K-steps land during this
//    unit's attention); rows >= L read row L-1 (finite, masked keys / unstored queries).
//  * LDS row = 64 B (4 chunks of 16 B), chunk XOR (row >> 1) & 3: conflict-free ds_read_b128
//    fragment reads of any 16-row block.
//  * units are dealt XCD by XCD in image-major order, so the 12 heads of an image run at about
//    the same time on one XCD and its token rows are read from HBM once (L2 shared).
constexpr int QA_KS = 32;     // K-step (halves): 64-byte LDS rows
constexpr int QA_NC = 192;    // q | k | v columns of one head
constexpr int QA_STAGES = 3;

__device__ __forceinline__ int qa_swz(int r, int c) { return r * QA_KS + ((c ^ ((r >> 1) & 3)) << 3); }

// LDS reads of an LDS-DMA'd slot by inline asm: hipcc would put a vmcnt(0) in front of a plain
// read of such a slot, draining the operand DMA in flight (the slot's own DMA is retired by the
// K-loop's counted wait + barrier).  Completed by the caller's lgkmcnt wait.
__device__ __forceinline__ f32x4 lds_read_f4(const float* p) {
    f32x4 v;
    asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"((uint32_t)(uintptr_t)(const __attribute__((address_space(3))) float*)p)
                 : "memory");
    return v;
}
// 0, but not known to the compiler (an inline-asm VGPR operand; inside a __device__ function,
// since the host pass instantiates __global__ template bodies and rejects the "v" constraint)
__device__ __forceinline__ int opaque_zero() {
    int z = 0;
    asm volatile("" : "+v"(z));
    return z;
}

__device__ __forceinline__ void lds_write_u2(void* p, uint2 v) {
    asm volatile("ds_write_b64 %0, %1" ::"v"(lds_addr(p)), "v"(v) : "memory");
}
__device__ __forceinline__ void lds_write_h(void* p, _Float16 v) {
    asm volatile("ds_write_b16 %0, %1" ::"v"(lds_addr(p)), "v"(v) : "memory");
}
__device__ __forceinline__ f16x8 lds_read_h8(const void* p) {
    f16x8 v;
    asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(lds_addr(p)) : "memory");
    return v;
}
// The wait that completes inline-asm LDS reads, with the read registers as operands: the
// compiler then cannot schedule a use of them above it (the hardware does not track VGPRs
// written by an outstanding LDS read).
template <typename A, typename B>
__device__ __forceinline__ void lgkm_wait(A& a, B& b) {
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a), "+v"(b)::"memory");
}
template <typename A, typename B, typename C, typename D>
__device__ __forceinline__ void lgkm_wait(A& a, B& b, C& c, D& d) {
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a), "+v"(b), "+v"(c), "+v"(d)::"memory");
}

__device__ __forceinline__ f32x2v lds_read_f2(const float* p) {
    f32x2v v;
    asm volatile("ds_read_b64 %0, %1" : "=v"(v) : "v"((uint32_t)(uintptr_t)(const __attribute__((address_space(3))) float*)p)
                 : "memory");
    return v;
}

#ifdef QA_DEBUG
__device__ _Float16 *g_dbg_q, *g_dbg_k, *g_dbg_vt;
__device__ int g_dbg_lp;
#endif

template <int NKB>
__global__ __launch_bounds__(NKB * 64, 1) void qkv_attn_kernel(const _Float16* __restrict__ x, int64_t ldx,
                                                               const _Float16* __restrict__ wq, int64_t ldw,
                                                               const float* __restrict__ bias,
                                                               const float* __restrict__ colsum,
                                                               const float2* __restrict__ rowstat, int L, int H, int Wd,
                                                               int64_t units, _Float16* __restrict__ o,
                                                               float scale_log2) {
    constexpr int R = NKB * 32;                       // padded token rows of an image
    constexpr int NW = NKB;                           // waves
    constexpr int SA = R * QA_KS;                     // A part of a stage (halves)
    constexpr int SS = (R + QA_NC) * QA_KS;           // one stage
    constexpr int APC = R / 16, PCS = APC + QA_NC / 16;  // 1 KiB DMA pieces per stage
    constexpr int PPW = (PCS + NW - 1) / NW;          // pieces per wave (uniform: extra ones repeat a W piece)
    constexpr int VS = R + 4;                         // v^T row stride (vt_stride)
    extern __shared__ __attribute__((aligned(16))) _Float16 lds[];
    _Float16* sK = lds + QA_STAGES * SS;
    _Float16* sV = sK + R * 64;
    // the unit's epilogue operands, DMA'd at its first K-step (a global load in the epilogue
    // would wait for the next unit's operand DMA issued before it: vmcnt retires in order):
    // bias [192] at +0, colsum [192] at +1 KiB, rowstat of the image's R rows at +2 KiB
    float* sE = (float*)(sV + 64 * VS);
    const int G = gridDim.x, bid = blockIdx.x;
    const int ng = G < 8 ? G : 8;
    const int xg = bid % ng;
    const int gx = G / ng + ((G % ng) > xg ? 1 : 0);
    const int64_t ulo = units * xg / ng, uhi = units * (xg + 1) / ng;
    const int64_t ufirst = ulo + bid / ng;
    if (ufirst >= uhi) return;
    const int nk = Wd / QA_KS;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);

    // DMA pieces of this wave (the same piece numbers every K-step): pc = wid + NW j; pieces
    // >= PCS repeat a W piece.  Per-lane source offsets (halves) from the unit's base are fixed.
    const int rp = lane >> 2;               // row inside the piece
    const int lch = (lane & 3) ^ ((rp >> 1) & 3);  // logical 16-byte chunk of the lane's physical one
    uint32_t boff[PPW];  // per-lane byte offset from the piece's wave-uniform source base
#pragma unroll
    for (int j = 0; j < PPW; j++) {
        int pc = wid + NW * j;
        if (pc >= PCS) pc = pc - PCS + APC;
        if (pc < APC) {
            const int r = pc * 16 + rp;
            boff[j] = (uint32_t)(((r < L ? r : L - 1) * (int)ldx + lch * 8) * 2);
        } else {
            const int jj = (pc - APC) * 16 + rp;
            boff[j] = (uint32_t)((((jj >> 6) * Wd + (jj & 63)) * (int)ldw + lch * 8) * 2);
        }
    }
    struct Pos {
        int64_t unit;
        int kt;
        const _Float16* xb;  // x rows of the unit's image
        const _Float16* wb;  // the unit's head rows of wq
    };
    auto set_unit = [&](Pos& p, int64_t u) {
        p.unit = u;
        p.kt = 0;
        const int64_t b = u / H;
        p.xb = x + b * L * ldx;
        p.wb = wq + (u - b * H) * 64 * ldw;
    };
    auto adv = [&](Pos& p) {
        if (++p.kt == nk) set_unit(p, p.unit + gx);
    };
    auto issue = [&](const Pos& p, int stage) {
        _Float16* st = lds + stage * SS;
#pragma unroll
        for (int j = 0; j < PPW; j++) {
            int pc = wid + NW * j;  // wave-uniform
            if (pc >= PCS) pc = pc - PCS + APC;
            const bool a = pc < APC;
            const char* base = (const char*)((a ? p.xb : p.wb) + p.kt * QA_KS);
            // (a void* source: with a char* the host pass drops the kernel's instantiation)
            __builtin_amdgcn_global_load_lds((const void*)(base + boff[j]),
                                             (lds_ptr_t)(st + (a ? pc * 512 : SA + (pc - APC) * 512)), 16, 0, 0);
        }
    };
    // one epilogue-operand DMA per wave per unit: wave 1 colsum, waves 2 / 3 the rowstat rows,
    // the others the bias (lanes 0-15 q, 16-31 k, 32-47 v columns of the head; waves past 3
    // repeat wave 0's piece: same bytes, same place)
    const uint32_t eoff = wid == 2 || wid == 3
                              ? (uint32_t)(((wid - 2) * 256 + lane * 4) * 4)
                              : (uint32_t)(((lane >> 4 < 3 ? lane >> 4 : 2) * Wd + (lane & 15) * 4) * 4);
    auto issue_epi = [&](int64_t u, int z) {
        const uint32_t eo = eoff + (uint32_t)z;
        const int64_t b = u / H;
        const int h = (int)(u - b * H);
        if (wid == 2 || wid == 3) {
            __builtin_amdgcn_global_load_lds((const void*)((const char*)(rowstat + b * L) + eo),
                                             (lds_ptr_t)(sE + 512 + (wid - 2) * 256), 16, 0, 0);
        } else {
            const float* v = wid == 1 ? colsum : bias;
            __builtin_amdgcn_global_load_lds((const void*)((const char*)(v + h * 64) + eo),
                                             (lds_ptr_t)(sE + (wid == 1 ? 256 : 0)), 16, 0, 0);
        }
    };

    f32x4 acc[2][12];
    Pos pd;  // next DMA position
    set_unit(pd, ufirst);
    int stage_d = 0;
    issue(pd, 0);
    adv(pd);
    if (pd.unit < uhi) issue(pd, 1);
    adv(pd);
    stage_d = 2;
    int stage_c = 0;
    for (int64_t u = ufirst; u < uhi; u += gx) {
        const int64_t b = u / H;
        const int h = (int)(u - b * H);  // (one division per unit)
        // an opaque zero offset: keeps the epilogue's and the attention's LDS / DMA address
        // arithmetic inside the unit loop (hoisted, it held ~30 VGPRs through the K-loop and
        // forced spills, whose reloads wait for every DMA in flight)
        const int z = opaque_zero();
#pragma unroll
        for (int i = 0; i < 2; i++)
#pragma unroll
            for (int j = 0; j < 12; j++) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int kt = 0; kt < nk; kt++) {
            // this step's DMA landed (the next step's stays in flight; at step 1 also the
            // epilogue-operand DMA issued between them), then every wave's
            if (kt == 1)
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PPW + 1) : "memory");
            else if (kt + 1 < nk || u + gx < uhi)
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PPW) : "memory");
            else
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            // ... and every wave is past the step that read the stage refilled here (and, at
            // step 0, past the previous unit's epilogue, which read the epilogue slot)
            if (kt == 0) issue_epi(u, z);
            if (pd.unit < uhi) {
                issue(pd, stage_d);
                adv(pd);
                stage_d = stage_d == QA_STAGES - 1 ? 0 : stage_d + 1;
            }
            const _Float16* sA = lds + stage_c * SS;
            const _Float16* sW = sA + SA;
            // all 14 fragments in flight before the MFMAs (the compiler would otherwise wait
            // for each W fragment right before its pair of MFMAs)
            f16x8 af[2], wf[12];
#pragma unroll
            for (int i = 0; i < 2; i++) af[i] = *(const f16x8*)(sA + qa_swz(wid * 32 + i * 16 + (lane & 15), lane >> 4));
#pragma unroll
            for (int j = 0; j < 12; j++) wf[j] = *(const f16x8*)(sW + qa_swz(j * 16 + (lane & 15), lane >> 4));
#pragma unroll
            for (int j = 0; j < 12; j++)
#pragma unroll
                for (int i = 0; i < 2; i++)
#ifndef QA_NO_MFMA  // timing variants (tools/qkv_attn_ab.py)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf[j], af[i], acc[i][j], 0, 0, 0);
#else
                    acc[i][j] += f32x4{(float)wf[j][0], (float)af[i][0], 0.f, 0.f};
#endif
            __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);  // 8 fragment reads
#pragma unroll
            for (int g = 0; g < 6; g++) {
                __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);  // 2 MFMAs
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // 1 read
            }
            __builtin_amdgcn_sched_group_barrier(0x008, 12, 0);
            stage_c = stage_c == QA_STAGES - 1 ? 0 : stage_c + 1;
        }
        // ---- epilogue: ln_1 fold + bias (gemm.hip), fp16 q / k / v (RNE)
        const int q4 = lane >> 4;
        f32x2v rs[2];
#pragma unroll
        for (int i = 0; i < 2; i++) {
            const int t = wid * 32 + i * 16 + (lane & 15);
            rs[i] = lds_read_f2(sE + z + 512 + 2 * (t < L ? t : L - 1));
        }
        lgkm_wait(rs[0], rs[1]);
        auto fold = [&](int j) {
            const int c = j * 16 + 4 * q4;  // column of the unit's 192
            f32x4 bn = lds_read_f4(sE + z + c), sn = lds_read_f4(sE + z + 256 + c);
            lgkm_wait(bn, sn);
#pragma unroll
            for (int i = 0; i < 2; i++) {
                acc[i][j][0] = __builtin_fmaf(rs[i].x, acc[i][j][0], __builtin_fmaf(rs[i].y, sn.x, bn.x));
                acc[i][j][1] = __builtin_fmaf(rs[i].x, acc[i][j][1], __builtin_fmaf(rs[i].y, sn.y, bn.y));
                acc[i][j][2] = __builtin_fmaf(rs[i].x, acc[i][j][2], __builtin_fmaf(rs[i].y, sn.z, bn.z));
                acc[i][j][3] = __builtin_fmaf(rs[i].x, acc[i][j][3], __builtin_fmaf(rs[i].y, sn.w, bn.w));
            }
        };
        _Float16* qs = sV + z + wid * (32 * 64);  // this wave's q rows, staged in the v^T region
#pragma unroll
        for (int j = 0; j < 8; j++) {
            fold(j);
#pragma unroll
            for (int i = 0; i < 2; i++) {
                const int tl = i * 16 + (lane & 15);
                const uint2 pk = make_uint2(cvt_pk_h(acc[i][j][0], acc[i][j][1]), cvt_pk_h(acc[i][j][2], acc[i][j][3]));
                if (j < 4) {
                    lds_write_u2(qs + tl * 64 + j * 16 + 4 * q4, pk);
                } else {
                    const int t = wid * 32 + tl, d0 = (j - 4) * 16 + 4 * q4;
                    lds_write_u2(sK + z + kswz(t, d0 >> 3) + (d0 & 7), pk);
                }
            }
        }
#pragma unroll
        for (int j = 8; j < 12; j++) fold(j);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#ifdef QA_DEBUG
        // debug tap: the folded q / k / v^T in the unfused layouts
        if (g_dbg_q) {
            for (int i = 0; i < 2; i++)
                for (int j = 0; j < 12; j++) {
                    const int t = wid * 32 + i * 16 + (lane & 15);
                    if (t >= L) continue;
                    for (int e = 0; e < 4; e++) {
                        const int c = j * 16 + 4 * q4 + e;
                        const _Float16 v = (_Float16)acc[i][j][e];
                        if (c < 64) g_dbg_q[(u * L + t) * 64 + c] = v;
                        else if (c < 128) g_dbg_k[(u * L + t) * 64 + c - 64] = v;
                        else g_dbg_vt[(u * 64 + c - 128) * (int64_t)g_dbg_lp + t] = v;
                    }
                }
        }
#endif
        f16x8 qf[4];
        {
            const int tl = lane & 31, hh = lane >> 5;
#pragma unroll
            for (int ks = 0; ks < 4; ks++) qf[ks] = lds_read_h8(qs + tl * 64 + ks * 16 + hh * 8);
            lgkm_wait(qf[0], qf[1], qf[2], qf[3]);
        }
        __builtin_amdgcn_s_barrier();  // every wave has its q: the v^T region is free
#pragma unroll
        for (int j = 8; j < 12; j++)
#pragma unroll
            for (int i = 0; i < 2; i++) {
                const int t = wid * 32 + i * 16 + (lane & 15), d0 = (j - 8) * 16 + 4 * q4;
#pragma unroll
                for (int e = 0; e < 4; e++)
                    lds_write_h(sV + z + (d0 + e) * VS + t, t < L ? f32_to_h(acc[i][j][e]) : (_Float16)0.0f);
            }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
#ifndef QA_NO_ATTN
        attn_block<NKB, false>(sK + z, sV + z, VS, qf, wid * 32 + (lane & 31), L, u, H, o, scale_log2);
#else
        if (lane == 0 && wid == 0) o[u] = qf[0][0] + sK[z + lane] + sV[z + 5];
#endif
    }
}

// V^T row stride (elements): LP + 4, i.e. LP/2 + 2 dwords, which is 2 mod 4 dwords (LP is a
// multiple of 32): the 32 rows of one half-wave ds_read_b64 then start on 32 distinct even
// banks (row r at bank 2 * (r * odd mod 32)), so they cover all 64 banks exactly once.  (The
// stride 2 mod 64 used before padded V^T by up to 60 elements per row: 23 % of V at L = 211.)
// The QKV epilogue writes V^T with this same stride in HBM, so one head's V^T is a contiguous
// blob for the LDS-DMA copy; 64 * (LP + 4) * 2 bytes is a multiple of 512.
#endif  // REIDMI_TOOLS (fused QKV GEMM + attention kernel)

static int vt_stride(int lp) { return lp + 4; }

static int g_num_cu = 0;
static int num_cu() {
    if (!g_num_cu) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&g_num_cu, hipDeviceAttributeMultiprocessorCount, dev);
        if (g_num_cu <= 0) g_num_cu = 256;
    }
    return g_num_cu;
}

template <int NKB>
static int launch_mhsa_pipe(const void* q, const void* k, const void* vt, void* o, int64_t nseq, int L, int H,
                            hipStream_t s) {
    constexpr int LP = NKB * 32, VS = LP + 4;
    const size_t lds = 2 * ((size_t)LP * 64 * 2 + (size_t)64 * VS * 2);
    static bool attr = false;
    if (!attr) {
        RM_CHECK_HIP(hipFuncSetAttribute((const void*)mhsa_pipe_kernel<NKB>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                         (int)lds));
        attr = true;
    }
    const int64_t nbh = nseq * H;
    static int occ = 0;
    if (!occ) {
        int n = 0;
        RM_CHECK_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, (const void*)mhsa_pipe_kernel<NKB>, NKB * 64, lds));
        occ = n > 0 ? n : 1;
    }
    const int64_t slots = (int64_t)num_cu() * occ;
    const int64_t grid = nbh < slots ? nbh : slots;
    hipLaunchKernelGGL((mhsa_pipe_kernel<NKB>), dim3((unsigned)grid), dim3(NKB * 64), lds, s, (const _Float16*)q,
                       (const _Float16*)k, (const _Float16*)vt, (_Float16*)o, L, H, nbh,
                       0.125f * 1.4426950408889634f);
    RM_LAUNCHED();
    return OK;
}

#ifdef REIDMI_TOOLS
static int launch_mhsa_rr(const void* q, const void* k, const void* vt, void* o, int64_t nseq, int L, int H,
                          hipStream_t s) {
    constexpr int NKB = 7, VS = kRrVS;
    // three slots + the overhang of the last slot's masked V^T reads (< 32 halves)
    constexpr size_t lds = (size_t)kRrSlots * (VS * 64 + 64 * VS) * 2 + 64;
    static_assert(lds <= 160 * 1024, "three slots must fit the CU's LDS");
    auto kern = mhsa_rr_kernel<NKB, VS>;
    static bool attr = false;
    if (!attr) {
        RM_CHECK_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        attr = true;
    }
    const int64_t nbh = nseq * H;  // < 2^31 (mhsa)
    const int64_t grid = nbh < num_cu() ? nbh : num_cu();  // one workgroup per CU (LDS)
    hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(kRrWaves * 64), lds, s, (const _Float16*)q,
                       (const _Float16*)k, (const _Float16*)vt, (_Float16*)o, L, H, nbh, 0.125f * 1.4426950408889634f);
    RM_LAUNCHED();
    return OK;
}
#endif  // REIDMI_TOOLS

template <int NKB, bool CAUSAL>
static int launch_mhsa(const void* q, const void* k, const void* vt, void* o, int64_t nseq, int L, int H,
                       int lpad_g, hipStream_t s) {
    if constexpr (!CAUSAL && ATTN_PIPE) {
        RM_REQUIRE(lpad_g == vt_stride(NKB * 32), "mhsa: v^T row stride must be reidmi_attn_lpad(L)");
        return launch_mhsa_pipe<NKB>(q, k, vt, o, nseq, L, H, s);
    } else {  // (discarded for the pipelined shapes: mhsa_kernel<NKB, false> is not instantiated)
    constexpr int LP = NKB * 32;
    // three LDS stages for the short causal (text) shapes (mhsa_kernel NS), two otherwise
    constexpr int NS = CAUSAL && NKB <= 4 ? ATTN_TEXT_STAGES : 2;
    const int vs = vt_stride(LP);
    RM_REQUIRE(lpad_g == vs, "mhsa: v^T row stride must be reidmi_attn_lpad(L)");
    RM_REQUIRE(NS == 2 || (vs == LP + 4 && (L + 31) / 32 == NKB), "mhsa: ring counts assume V^T rows of LP + 4");
    const size_t stage = (size_t)LP * 64 * 2 + (size_t)64 * vs * 2;
    const size_t lds = NS * stage;
    const float scale_log2 = 0.125f * 1.4426950408889634f;  // 1/sqrt(64) * log2(e)
    auto kern = mhsa_kernel<NKB, CAUSAL, NS>;
    static bool attr = false;
    if (!attr) {
        RM_CHECK_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        attr = true;
    }
    const int64_t nbh = nseq * H;
    const int waves = (L + 31) / 32;
    // Persistent grid: as many workgroups per CU as fit (LDS, VGPRs).  Vision (L = 211: 7
    // waves, 2 x 57 KB LDS) fits one; short text rows (L <= 64: 2 waves, 2 x 17 KB) fit four,
    // which a single workgroup per CU would leave latency-bound on its K/V loads.
    static int occ_waves = -1, occ = 1;
    if (occ_waves != waves) {
        int n = 0;
        RM_CHECK_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, (const void*)kern, 64 * waves, lds));
        occ = n > 0 ? n : 1;
        occ_waves = waves;
    }
    const int64_t slots = (int64_t)num_cu() * occ;
    const int64_t grid = nbh < slots ? nbh : slots;
    hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(64 * waves), lds, s,
                       (const _Float16*)q, (const _Float16*)k, (const _Float16*)vt, (_Float16*)o, L, H, vs, nbh,
                       scale_log2);
    RM_LAUNCHED();
    return OK;
    }
}

// CLS query only (the last block of the inference path): one wave per (sequence, head).
// q [nseq*H][64] (the CLS rows), k [nseq*H][L][64], vt [nseq*H][64][lpad] -> o [nseq][H*64].
// Lane t-strided scores, wave-reduced softmax, probabilities through LDS, lane d sums
// p_t * V^T[d][t] over its contiguous row.
__global__ __launch_bounds__(256) void mhsa_cls_kernel(const _Float16* __restrict__ q, const _Float16* __restrict__ k,
                                                       const _Float16* __restrict__ vt, _Float16* __restrict__ o,
                                                       int64_t nbh, int L, int H, int lpad, float scale_log2) {
    __shared__ float sp[4][256];
    __shared__ float sq[4][64];
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t bh = (int64_t)blockIdx.x * 4 + wid;
    if (bh >= nbh) return;
    sq[wid][lane] = (float)q[bh * 64 + lane];
    __builtin_amdgcn_wave_barrier();
    const _Float16* kh = k + bh * (int64_t)L * 64;
    float sv[4];
    float mx = -__builtin_inff();
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const int t = lane + 64 * j;
        float a = -__builtin_inff();
        if (t < L) {
            a = 0.f;
            const f16x8* kr = (const f16x8*)(kh + (int64_t)t * 64);
#pragma unroll
            for (int c = 0; c < 8; c++) {
                const f16x8 kv = kr[c];
#pragma unroll
                for (int e = 0; e < 8; e++) a += sq[wid][c * 8 + e] * (float)kv[e];
            }
            a *= scale_log2;
        }
        sv[j] = a;
        mx = fmaxf(mx, a);
    }
    mx = wave_max(mx);
    float sum = 0.f;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const int t = lane + 64 * j;
        const float p = t < L ? __builtin_amdgcn_exp2f(sv[j] - mx) : 0.f;
        // fp16-rounded probabilities, as the blocked kernel feeds its P.V MFMAs
        sp[wid][t] = (float)(_Float16)p;
        sum += p;
    }
    sum = wave_sum(sum);
    __builtin_amdgcn_wave_barrier();
    // lane d: p . V^T[d][:].  All row loads are issued before the first use (a rolled loop
    // waited one HBM round trip per 8 keys); same summation order as before.
    const _Float16* vr = vt + (bh * 64 + lane) * (int64_t)lpad;
    f16x8 vv[32];
#pragma unroll
    for (int i = 0; i < 32; i++)
        if (i * 8 < L) vv[i] = *(const f16x8*)(vr + i * 8);
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < 32; i++)
        if (i * 8 < L)
#pragma unroll
            for (int e = 0; e < 8; e++)
                if (i * 8 + e < L) acc += sp[wid][i * 8 + e] * (float)vv[i][e];
    const int64_t b = bh / H, h = bh % H;
    o[b * (int64_t)H * 64 + h * 64 + lane] = (_Float16)(acc / sum);
}

int mhsa_cls(const void* q, const void* k, const void* vt, void* o, int64_t nseq, int L, int H, hipStream_t s) {
    const int lp = attn_lpad(L);
    RM_REQUIRE(lp > 0, "mhsa_cls: sequence length must be <= 256");
    const int64_t nbh = nseq * H;
    hipLaunchKernelGGL(mhsa_cls_kernel, dim3(ceil_div(nbh, 4)), dim3(256), 0, s, (const _Float16*)q, (const _Float16*)k,
                       (const _Float16*)vt, (_Float16*)o, nbh, L, H, lp, 0.125f * 1.4426950408889634f);
    RM_LAUNCHED();
    return OK;
}

// ------------------------------------------------- the last block's CLS attention without K, V
// Only the CLS query's attention output is consumed in the last block (zero_shot_learning.py:
// 85-87 reads x12[:, 0] / xproj[:, 0]).  With the ln_1 fold (gemm.h: W' = W diag(gamma), s its
// column sums, b' = b + W beta, per row rstd_t and a_t = -mean_t rstd_t), key and value of token t
// are k_t = rstd_t (x_t W_K'^T) + a_t s_K + b_K' and v_t alike, so for the CLS query q_h of head h
//   q_h . k_t = rstd_t (x_t . u_h) + a_t (q_h . s_Kh) + q_h . b_Kh',        u_h = W_Kh'^T q_h
//   sum_t p_t v_t = W_Vh' z_h + alpha_h s_Vh + b_Vh',  z_h = sum_t p_t rstd_t x_t,
//                                                      alpha_h = sum_t p_t a_t  (sum_t p_t = 1)
// (custom_clip_model.py:22-24 -> F.multi_head_attention_forward's in_proj + SDPA, reassociated):
// the same function of x without K and V for every token — 2 x 768 x 768 MACs per token and
// 2 x 324 KB of K / V^T per image never formed.  Unlike the K / V path, nothing in between is
// rounded to fp16 (u and the weights p rstd enter the MFMAs as fp16 hi + lo pairs, fp32-exact
// products), so the result is closer to the reference's fp32 run than the fp16 K / V it replaces.
//   cls_u_kernel     u_h (hi, lo), q_h . s_Kh, q_h . b_Kh' for 16 images per workgroup (VALU)
//   cls_attn_kernel  one image per workgroup: scores X u^T on MFMA, softmax, z = w^T X on MFMA
//                    (x staged in LDS and read transposed with ds_read_b64_tr_b16), alpha
//   cls_o_kernel     o = W_V' z + alpha s_V + b_V' -> fp16, 16 images per workgroup (VALU)
typedef __fp16 trh4 __attribute__((__vector_size__(8)));
constexpr int kClsImg = 16;  // images per workgroup of cls_u / cls_o
constexpr int kClsLp = 224;  // token rows covered by cls_attn (7 x 32): L <= 224

template <int W>
__global__ __launch_bounds__(256) void cls_u_kernel(const _Float16* __restrict__ q, const _Float16* __restrict__ wk,
                                                    const float* __restrict__ sk, const float* __restrict__ bk,
                                                    int64_t nseq, _Float16* __restrict__ u16, float* __restrict__ qsb) {
    constexpr int H = W / 64, J = W / 256, NP = kClsImg / 2;
    __shared__ f32x2v sq[W][NP];  // q[k] of the workgroup's images, as image pairs
    const int tid = threadIdx.x;
    const int64_t b0 = (int64_t)blockIdx.x * kClsImg;
    for (int e = tid; e < W * NP; e += 256) {
        const int k = e / NP, p = e - k * NP;
        const int64_t i0 = b0 + 2 * p;
        sq[k][p] = f32x2v{i0 < nseq ? (float)q[i0 * W + k] : 0.f, i0 + 1 < nseq ? (float)q[(i0 + 1) * W + k] : 0.f};
    }
    __syncthreads();
    if (tid < kClsImg * 16) {  // q_h . s_Kh and q_h . b_Kh' per (image, head)
        const int i = tid >> 4, h = tid & 15;
        float a = 0.f, c = 0.f;
        if (h < H)
            for (int d = 0; d < 64; d++) {
                const float qv = sq[64 * h + d][i >> 1][i & 1];
                a = __builtin_fmaf(qv, sk[64 * h + d], a);
                c = __builtin_fmaf(qv, bk[64 * h + d], c);
            }
        if (b0 + i < nseq && h < H) {
            qsb[(b0 + i) * 32 + h] = a;
            qsb[(b0 + i) * 32 + 16 + h] = c;
        }
    }
    for (int h = 0; h < H; h++) {
        f32x2v acc[NP][J];
#pragma unroll
        for (int p = 0; p < NP; p++)
#pragma unroll
            for (int j = 0; j < J; j++) acc[p][j] = f32x2v{0.f, 0.f};
        for (int d = 0; d < 64; d++) {
            const _Float16* wr = wk + (int64_t)(64 * h + d) * W;  // row 64h + d of W_K'
            float w[J];
#pragma unroll
            for (int j = 0; j < J; j++) w[j] = (float)wr[tid + 256 * j];
#pragma unroll
            for (int p = 0; p < NP; p++) {
                const f32x2v qq = sq[64 * h + d][p];
#pragma unroll
                for (int j = 0; j < J; j++) acc[p][j] = __builtin_elementwise_fma(qq, f32x2v{w[j], w[j]}, acc[p][j]);
            }
        }
#pragma unroll
        for (int p = 0; p < NP; p++)
#pragma unroll
            for (int e = 0; e < 2; e++) {
                const int64_t b = b0 + 2 * p + e;
                if (b >= nseq) continue;
#pragma unroll
                for (int j = 0; j < J; j++) {
                    const float v = acc[p][j][e];
                    const _Float16 hi = (_Float16)v;
                    const _Float16 lo = (_Float16)(v - (float)hi);
                    u16[((b * 2 + 0) * H + h) * (int64_t)W + tid + 256 * j] = hi;
                    u16[((b * 2 + 1) * H + h) * (int64_t)W + tid + 256 * j] = lo;
                }
            }
    }
}

// LDS of cls_attn_kernel: u (hi, lo) rows, one 32-token chunk of x rows, the 8 waves' partial
// scores, the chunk's weights p rstd (hi, lo), its row statistics, and per head the running
// max / normaliser / alpha and the chunk's rescale factor
template <int W>
struct ClsLds {
    static constexpr int US = W + 8, XS = W + 16, TS = 32 + 8;
    static constexpr int U_OFF = 0, X_OFF = U_OFF + 2 * 16 * US * 2, P_OFF = X_OFF + 32 * XS * 2;
    static constexpr int WT_OFF = P_OFF + 8 * 16 * 16 * 4, RS_OFF = WT_OFF + 2 * 16 * TS * 2;
    static constexpr int H_OFF = RS_OFF + 32 * 8, BYTES = H_OFF + 16 * 4 * 4;
};

// One image per workgroup, its tokens in 32-row chunks (online softmax, each x row read once):
// the chunk's x rows are staged in LDS (the next chunk's are loaded into registers meanwhile);
// scores D[h = 4g + e][t = l15] = u_h . x_t on MFMA (A = u rows, B = x rows), the two 16-token
// tiles split over the 8 waves by K quarters and summed by the softmax threads; per head the
// running max m, normaliser l and alpha are updated and the chunk's weights w_t = p_t rstd_t
// (hi, lo) written; z accumulates D[h][c] = sum_t w[h][t] x_t[c] on MFMA, its rows rescaled by
// exp2(m_old - m_new) (B = x columns read transposed: lane 4q + p of a 16-lane group addresses
// row q, columns 4p..4p+3 of a 4 x 16 block and receives column l15 of its 4 rows).
template <int W>
__global__ __launch_bounds__(512) void cls_attn_kernel(const _Float16* __restrict__ x, const float2* __restrict__ rs,
                                                       const _Float16* __restrict__ u16, const float* __restrict__ qsb,
                                                       int64_t nseq, int L, float scale_log2, float* __restrict__ z,
                                                       float* __restrict__ alpha) {
    constexpr int H = W / 64, KQ = W / 32 / 4, CT = W / 16 / 8;  // k-steps per quarter; z column tiles per wave
    constexpr int XV = 32 * (W / 8) / 512;                         // 16-byte pieces of a chunk per thread
    static_assert(32 * (W / 8) % 512 == 0, "chunk pieces per thread");
    using C = ClsLds<W>;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    _Float16* sU = (_Float16*)(smem + C::U_OFF);    // [2][16][US]
    _Float16* sX = (_Float16*)(smem + C::X_OFF);    // [32][XS]
    float* sP = (float*)(smem + C::P_OFF);          // [8 waves][16 h][16 t]
    _Float16* sWt = (_Float16*)(smem + C::WT_OFF);  // [2][16][TS]
    float2* sRS = (float2*)(smem + C::RS_OFF);      // [32]
    float* sH = (float*)(smem + C::H_OFF);          // [16] rescale factor, then [16] final 1 / l
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int l15 = lane & 15, g = lane >> 4;
    const int nch = (L + 31) / 32;
    for (int64_t b = blockIdx.x; b < nseq; b += gridDim.x) {
        const _Float16* xb = x + b * L * (int64_t)W;
        f16x8 xr[XV];
        auto fetch = [&](int ch) {  // piece e of the chunk: row e / (W/8), 16 bytes at column 8 (e % (W/8))
#pragma unroll
            for (int v = 0; v < XV; v++) {
                const int e = tid + 512 * v, r = e / (W / 8), c8 = e % (W / 8);
                const int t = ch * 32 + r < L ? ch * 32 + r : L - 1;  // (rows >= L carry weight 0)
                xr[v] = *(const f16x8*)(xb + (int64_t)t * W + c8 * 8);
            }
        };
        fetch(0);
        for (int e = tid; e < 2 * 16 * (W / 8); e += 512) {
            const int hl = e / (16 * (W / 8)), r = e / (W / 8) % 16, c8 = e % (W / 8);
            f16x8 v = {};
            if (r < H) v = *(const f16x8*)(u16 + ((b * 2 + hl) * H + r) * (int64_t)W + c8 * 8);
            *(f16x8*)(sU + (hl * 16 + r) * C::US + c8 * 8) = v;
        }
        // softmax state of head hs = tid / 32 (every thread of the head's 32 holds it)
        const int hs = tid >> 5, part = tid & 31;
        const float sig = hs < H ? qsb[b * 32 + hs] : 0.f, bet = hs < H ? qsb[b * 32 + 16 + hs] : 0.f;
        float m = -__builtin_inff(), l = 0.f, al = 0.f;
        f32x4 zacc[CT];
#pragma unroll
        for (int i = 0; i < CT; i++) zacc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int ch = 0; ch < nch; ch++) {
            __syncthreads();  // the previous chunk's readers of sX / sWt / sRS / sH are done
#pragma unroll
            for (int v = 0; v < XV; v++) {
                const int e = tid + 512 * v, r = e / (W / 8), c8 = e % (W / 8);
                *(f16x8*)(sX + r * C::XS + c8 * 8) = xr[v];
            }
            if (tid < 32) sRS[tid] = ch * 32 + tid < L ? rs[b * L + ch * 32 + tid] : make_float2(0.f, 0.f);
            if (ch + 1 < nch) fetch(ch + 1);
            __syncthreads();
            {  // partial scores: tile wid & 1 (tokens 16 (wid & 1) ..), K quarter wid >> 1
                const int tile = wid & 1, kq = wid >> 1;
                f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int k = 0; k < KQ; k++) {
                    const int c = (kq * KQ + k) * 32 + g * 8;
                    const f16x8 xf = *(const f16x8*)(sX + (tile * 16 + l15) * C::XS + c);
                    const f16x8 uh = *(const f16x8*)(sU + l15 * C::US + c);
                    const f16x8 ul = *(const f16x8*)(sU + (16 + l15) * C::US + c);
                    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(uh, xf, acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ul, xf, acc, 0, 0, 0);
                }
#pragma unroll
                for (int e = 0; e < 4; e++) sP[(wid * 16 + 4 * g + e) * 16 + l15] = acc[e];
            }
            __syncthreads();
            {  // online softmax of head hs over the chunk's token part
                const int t = ch * 32 + part, tile = part >> 4, tl = part & 15;
                float raw = 0.f;
#pragma unroll
                for (int kq = 0; kq < 4; kq++) raw += sP[((2 * kq + tile) * 16 + hs) * 16 + tl];
                const float2 st = sRS[part];
                const float sc = hs < H && t < L ? (st.x * raw + st.y * sig + bet) * scale_log2 : -__builtin_inff();
                float cm = sc;
#pragma unroll
                for (int o = 16; o >= 1; o >>= 1) cm = fmaxf(cm, __shfl_xor(cm, o, 32));
                const float mn = fmaxf(m, cm);
                const float f = hs < H ? __builtin_amdgcn_exp2f(m - mn) : 1.f;  // (m = -inf: 0)
                const float p = hs < H && t < L ? __builtin_amdgcn_exp2f(sc - mn) : 0.f;
                float ps = p, pa = p * st.y;
#pragma unroll
                for (int o = 16; o >= 1; o >>= 1) {
                    ps += __shfl_xor(ps, o, 32);
                    pa += __shfl_xor(pa, o, 32);
                }
                l = __builtin_fmaf(l, f, ps);
                al = __builtin_fmaf(al, f, pa);
                m = hs < H ? mn : m;
                const float w = p * st.x;
                const _Float16 hi = (_Float16)w;
                sWt[hs * C::TS + part] = hi;
                sWt[(16 + hs) * C::TS + part] = (_Float16)(w - (float)hi);
                if (part == 0) sH[hs] = f;
            }
            __syncthreads();
            {  // z: rescale, then + w^T x (hi, lo)
                float fr[4];
#pragma unroll
                for (int e = 0; e < 4; e++) fr[e] = sH[4 * g + e];
                const f16x8 ah = *(const f16x8*)(sWt + l15 * C::TS + g * 8);
                const f16x8 alo = *(const f16x8*)(sWt + (16 + l15) * C::TS + g * 8);
#pragma unroll
                for (int i = 0; i < CT; i++) {
                    const int c0 = (wid + 8 * i) * 16;
                    const _Float16* a0 = sX + (8 * g + (l15 >> 2)) * C::XS + c0 + 4 * (l15 & 3);
                    const trh4 r0 = __builtin_amdgcn_ds_read_tr16_b64_v4f16((__attribute__((address_space(3))) trh4*)a0);
                    const trh4 r1 = __builtin_amdgcn_ds_read_tr16_b64_v4f16(
                        (__attribute__((address_space(3))) trh4*)(a0 + 4 * C::XS));
                    const uint2 u0 = __builtin_bit_cast(uint2, r0), u1 = __builtin_bit_cast(uint2, r1);
                    const f16x8 bf = __builtin_bit_cast(f16x8, make_uint4(u0.x, u0.y, u1.x, u1.y));
#pragma unroll
                    for (int e = 0; e < 4; e++) zacc[i][e] *= fr[e];
                    zacc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bf, zacc[i], 0, 0, 0);
                    zacc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(alo, bf, zacc[i], 0, 0, 0);
                }
            }
        }
        __syncthreads();
        if (part == 0) sH[16 + hs] = hs < H ? 1.0f / l : 0.f;
        if (part == 0 && hs < H) alpha[b * H + hs] = al / l;
        __syncthreads();
        float inv[4];
#pragma unroll
        for (int e = 0; e < 4; e++) inv[e] = sH[16 + 4 * g + e];
#pragma unroll
        for (int i = 0; i < CT; i++) {
            const int c0 = (wid + 8 * i) * 16;
#pragma unroll
            for (int e = 0; e < 4; e++) {
                const int h = 4 * g + e;
                if (h < H) z[(b * H + h) * (int64_t)W + c0 + l15] = zacc[i][e] * inv[e];
            }
        }
    }
}

// o[b][n] = W_V'[n] . z[b][h(n)] + alpha[b][h] s_V[n] + b_V'[n] for 16 images per workgroup on
// MFMA: D[n = n0 + 4g + e][image = l15] over 16-row tiles of W_V' (A, rows straight from HBM)
// and the images' z rows (B, fp32 -> fp16 hi + lo: fp32-exact products)
template <int W>
__global__ __launch_bounds__(256) void cls_o_kernel(const float* __restrict__ z, const float* __restrict__ alpha,
                                                    const _Float16* __restrict__ wv, const float* __restrict__ sv,
                                                    const float* __restrict__ bv, int64_t nseq, _Float16* __restrict__ o) {
    constexpr int H = W / 64, KS = W / 32;
    const int lane = threadIdx.x & 63, l15 = lane & 15, g = lane >> 4;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t b0 = (int64_t)blockIdx.x * kClsImg;
    const int64_t img = b0 + l15 < nseq ? b0 + l15 : nseq - 1;  // (images past nseq: not stored)
    // a wave per head: its 4 N-tiles share the head's z fragment (loaded and split into fp16 hi / lo
    // once per K-step) and run 4 independent MFMA chains; each output's chain is unchanged
    for (int h = wid; h < H; h += 4) {
        const _Float16* wr = wv + (int64_t)(64 * h + l15) * W + g * 8;
        const float* zr = z + (img * H + h) * (int64_t)W + g * 8;
        f32x4 acc[4] = {};
#pragma unroll 2
        for (int ks = 0; ks < KS; ks++) {
            f16x8 a[4];
#pragma unroll
            for (int t = 0; t < 4; t++) a[t] = *(const f16x8*)(wr + (int64_t)t * 16 * W + ks * 32);
            const float4 z0 = *(const float4*)(zr + ks * 32), z1 = *(const float4*)(zr + ks * 32 + 4);
            const float zv[8] = {z0.x, z0.y, z0.z, z0.w, z1.x, z1.y, z1.z, z1.w};
            f16x8 bh, bl;
#pragma unroll
            for (int e = 0; e < 8; e++) {
                bh[e] = (_Float16)zv[e];
                bl[e] = (_Float16)(zv[e] - (float)bh[e]);
            }
#pragma unroll
            for (int t = 0; t < 4; t++) {
                acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[t], bh, acc[t], 0, 0, 0);
                acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[t], bl, acc[t], 0, 0, 0);
            }
        }
        if (b0 + l15 < nseq) {
            const float al = alpha[img * H + h];
#pragma unroll
            for (int t = 0; t < 4; t++) {
                const int n0 = 64 * h + 16 * t;
                _Float16 r[4];
#pragma unroll
                for (int e = 0; e < 4; e++) {
                    const int n = n0 + 4 * g + e;
                    r[e] = (_Float16)(acc[t][e] + al * sv[n] + bv[n]);
                }
                *(uint2*)(o + img * W + n0 + 4 * g) = __builtin_bit_cast(uint2, r);
            }
        }
    }
}

int64_t cls_attn_nokv_ws_bytes(int64_t nseq, int W) {
    const int64_t H = W / 64;
    auto al = [](int64_t v) { return (v + 255) / 256 * 256; };
    return al(nseq * 2 * H * W * 2) + al(nseq * 32 * 4) + al(nseq * H * W * 4) + al(nseq * H * 4);
}

template <int W>
static int launch_cls_nokv(const _Float16* x, const float2* rs, const _Float16* q, const _Float16* wqkv,
                           const float* colsum, const float* bias, int64_t nseq, int L, char* ws, _Float16* o,
                           hipStream_t s) {
    constexpr int H = W / 64;
    auto al = [](int64_t v) { return (v + 255) / 256 * 256; };
    _Float16* u16 = (_Float16*)ws;
    float* qsb = (float*)(ws + al(nseq * 2 * H * W * 2));
    float* z = (float*)((char*)qsb + al(nseq * 32 * 4));
    float* alpha = (float*)((char*)z + al(nseq * H * W * 4));
    const unsigned nb = (unsigned)((nseq + kClsImg - 1) / kClsImg);
    hipLaunchKernelGGL(cls_u_kernel<W>, dim3(nb), dim3(256), 0, s, q, wqkv + (int64_t)W * W, colsum + W, bias + W, nseq,
                       u16, qsb);
    RM_LAUNCHED();
    static bool attr = false;
    static int occ = 0;
    if (!attr) {
        RM_CHECK_HIP(hipFuncSetAttribute((const void*)cls_attn_kernel<W>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                         ClsLds<W>::BYTES));
        int n = 0;
        RM_CHECK_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, (const void*)cls_attn_kernel<W>, 512,
                                                                  ClsLds<W>::BYTES));
        occ = n > 0 ? n : 1;
        attr = true;
    }
    const int64_t slots = (int64_t)num_cu() * occ;
    hipLaunchKernelGGL(cls_attn_kernel<W>, dim3((unsigned)(nseq < slots ? nseq : slots)), dim3(512), ClsLds<W>::BYTES, s,
                       x, rs, (const _Float16*)u16, (const float*)qsb, nseq, L, 0.125f * 1.4426950408889634f, z, alpha);
    RM_LAUNCHED();
    hipLaunchKernelGGL(cls_o_kernel<W>, dim3(nb), dim3(256), 0, s, (const float*)z, (const float*)alpha,
                       wqkv + (int64_t)2 * W * W, colsum + 2 * W, bias + 2 * W, nseq, o);
    RM_LAUNCHED();
    return OK;
}

// x [nseq*L][W] fp16 (the residual stream), rs [nseq*L] (rstd, -mean rstd) of its rows, q
// [nseq][W] fp16 (the CLS rows' heads, head-major), wqkv / colsum / bias the ln_1-folded in_proj
// ([3W][W] fp16, [3W], [3W]), ws >= cls_attn_nokv_ws_bytes -> o [nseq][W] fp16.
int cls_attn_nokv(const void* x, const void* rs, const void* q, const void* wqkv, const float* colsum,
                  const float* bias, int64_t nseq, int L, int H, int W, void* ws, void* o, hipStream_t s) {
    RM_REQUIRE(H * 64 == W && (W == 768 || W == 1024), "cls_attn_nokv: width 768 or 1024, 64-wide heads");
    RM_REQUIRE(L >= 1 && L <= kClsLp, "cls_attn_nokv: 1 <= L <= 224");
    if (nseq <= 0) return OK;
    auto f = W == 768 ? launch_cls_nokv<768> : launch_cls_nokv<1024>;
    return f((const _Float16*)x, (const float2*)rs, (const _Float16*)q, (const _Float16*)wqkv, colsum, bias, nseq, L,
             (char*)ws, (_Float16*)o, s);
}

#ifdef REIDMI_TOOLS
// Fused QKV + attention for non-causal blocks of L in (192, 224] tokens (the vision towers:
// 211, IVLP 213); returns EINVAL for other shapes (the caller then runs the two kernels).
// x [nseq*L][ldx] fp16 (the residual stream), wq [3W][ldw] fp16 (ln_1-folded in_proj), bias /
// colsum [3W] fp32, rowstat [nseq*L (+pad)] (rstd, -mean*rstd), o [nseq*L][W] fp16.
bool qkv_attn_fits(int L, int W, bool causal) { return !causal && L > 192 && L <= 224 && W % QA_KS == 0 && W >= 64; }

int qkv_attn(const void* x, int64_t ldx, const void* wq, int64_t ldw, const float* bias, const float* colsum,
             const void* rowstat, int64_t nseq, int L, int H, int W, void* o, hipStream_t s) {
    RM_REQUIRE(qkv_attn_fits(L, W, false) && W == H * 64 && nseq >= 0, "qkv_attn: shape");
    RM_REQUIRE(bias && colsum && rowstat && ldx >= W && ldw >= W && ldx % 8 == 0 && ldw % 8 == 0, "qkv_attn: args");
    const int64_t units = nseq * H;
    if (units == 0) return OK;
    RM_REQUIRE(units < (1ll << 31), "qkv_attn: too many units");
    constexpr int NKB = 7, R = NKB * 32;
    const size_t lds = ((size_t)QA_STAGES * (R + QA_NC) * QA_KS + (size_t)R * 64 + (size_t)64 * (R + 4)) * 2 + 4096;
    static bool attr = false;
    if (!attr) {
        RM_CHECK_HIP(hipFuncSetAttribute((const void*)qkv_attn_kernel<NKB>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                         (int)lds));
        attr = true;
    }
    const int64_t grid = units < num_cu() ? units : num_cu();
    hipLaunchKernelGGL((qkv_attn_kernel<NKB>), dim3((unsigned)grid), dim3(NKB * 64), lds, s, (const _Float16*)x, ldx,
                       (const _Float16*)wq, ldw, bias, colsum, (const float2*)rowstat, L, H, W, units, (_Float16*)o,
                       0.125f * 1.4426950408889634f);
    RM_LAUNCHED();
    return OK;
}
#endif  // REIDMI_TOOLS

// Smallest instantiated key-padding >= L.  Lp must also equal the vt row length the
// QKV epilogue wrote (attn_lpad()).
int attn_lpad(int L) {
    if (L < 1 || L > 256) return -1;
    return vt_stride((L + 31) / 32 * 32);  // row stride of V^T (elements), >= L
}

int mhsa(const void* q, const void* k, const void* vt, void* o, int64_t nseq, int L, int H, bool causal,
         hipStream_t s) {
    const int lp = attn_lpad(L);
    RM_REQUIRE(lp > 0, "mhsa: sequence length must be <= 256");
    RM_REQUIRE(nseq * H < (1ll << 31), "mhsa: too many (sequence, head) pairs");
#define RM_MHSA_CASE(n)                                                                                  \
    case n:                                                                                              \
        return causal ? launch_mhsa<n, true>(q, k, vt, o, nseq, L, H, lp, s)                            \
                      : launch_mhsa<n, false>(q, k, vt, o, nseq, L, H, lp, s);
    switch ((L + 31) / 32) {
        RM_MHSA_CASE(1)
        RM_MHSA_CASE(2)
        RM_MHSA_CASE(3)
        RM_MHSA_CASE(4)
        RM_MHSA_CASE(5)
        RM_MHSA_CASE(6)
        RM_MHSA_CASE(7)
        RM_MHSA_CASE(8)
    }
#undef RM_MHSA_CASE
    return fail(EINVAL_, "mhsa: unsupported length");
}

}  // namespace reidmi

using namespace reidmi;

REIDMI_API int reidmi_attn_lpad(int L) { return attn_lpad(L); }

#ifdef ATTN_STAMPS
REIDMI_API int reidmi_attn_stamps(uint64_t* host) {
    RM_CHECK_HIP(hipMemcpyFromSymbol(host, HIP_SYMBOL(g_attn_stamps), sizeof(g_attn_stamps)));
    return OK;
}
#endif

#ifdef QA_DEBUG
REIDMI_API int reidmi_qa_dbg_set(void* q, void* k, void* vt, int lp) {
    RM_CHECK_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_dbg_q), &q, sizeof(q)));
    RM_CHECK_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_dbg_k), &k, sizeof(k)));
    RM_CHECK_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_dbg_vt), &vt, sizeof(vt)));
    RM_CHECK_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_dbg_lp), &lp, sizeof(lp)));
    return OK;
}
#endif

REIDMI_API int reidmi_mhsa_f16(const void* q, const void* k, const void* vt, void* o, int64_t nseq, int L, int H,
                                int causal, void* stream) {
    return mhsa(q, k, vt, o, nseq, L, H, causal != 0, (hipStream_t)stream);
}

#ifdef REIDMI_TOOLS
// mhsa_rr_kernel (8 waves on round-robin (head, 32-query block) units, three LDS slots) for
// non-causal L in 205..212 with V^T rows of 212: the round-6 A/B of the product's two-stage
// kernel, bit-identical to it (tests/test_gpu_encoder.py, tools/attn_rr_ab.py).
REIDMI_API int reidmi_mhsa_f16_rr(const void* q, const void* k, const void* vt, void* o, int64_t nseq, int L, int H,
                                  void* stream) {
    RM_REQUIRE(L >= kRrLmin && L <= kRrVS && nseq * H < (1ll << 31), "reidmi_mhsa_f16_rr: 205 <= L <= 212");
    return launch_mhsa_rr(q, k, vt, o, nseq, L, H, (hipStream_t)stream);
}
#endif
