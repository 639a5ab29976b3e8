// attention.hip — fused multi-head self-attention for the CLIP encoders (gfx950).
//
// softmax(Q K^T / sqrt(64) [+ causal mask]) V for every (sequence, head), the SDPA that
// nn.MultiheadAttention dispatches in custom_clip_model.py:12,22-24 (vision: L = 211/213,
// no mask) and maple.py:956-962,976 (text: L = 77, additive -inf causal mask).
//
// One workgroup (4 waves) per (sequence, head).  K [Lp][64] and V^T [64][Lp] of the head
// live in LDS for the whole sweep (L <= 256 fits: one key sweep, no online rescaling).
// Each wave takes 16-query blocks:
//   S^T = K Q^T with v_mfma_f32_16x16x32_bf16 (K fragment as A) so each lane holds the
//     scores of ONE query for 4 keys per 16-key block -> row max / row sum are in-lane
//     plus two xor-shuffles across the 4 lane groups;
//   O^T = V^T P^T: the probabilities are already in the B-operand layout (the k order
//     inside each 32-key step is permuted identically on both operands), V^T rows are
//     read as 2 x 8 B from LDS.  O comes out one query per lane, 4 consecutive dims.
// Inputs from the QKV GEMM epilogue: q,k [B*H][L][64] bf16, vt [B*H][64][Lp] bf16.
// Output o [B*L][H*64] bf16 (token-major: the A operand of out_proj).
#include "common.h"

namespace reidmi {

__device__ __forceinline__ int kswz(int r, int kc) { return r * 64 + ((kc ^ ((r >> 1) & 7)) << 3); }

template <int NKB, bool CAUSAL>
__global__ __launch_bounds__(256) void mhsa_kernel(const __bf16* __restrict__ q, const __bf16* __restrict__ k,
                                                   const __bf16* __restrict__ vt, __bf16* __restrict__ o, int L,
                                                   int H, int lpad_g, int vstride, float scale_log2) {
    constexpr int LP = NKB * 16;
    extern __shared__ __attribute__((aligned(16))) __bf16 lds[];
    __bf16* sK = lds;                 // [LP][64], swizzled 16-byte chunks
    __bf16* sV = lds + LP * 64;       // [64][vstride]
    const int bh = blockIdx.x;
    const int b = bh / H, h = bh % H;
    const __bf16* qh = q + (int64_t)bh * L * 64;
    const __bf16* kh = k + (int64_t)bh * L * 64;
    const __bf16* vh = vt + (int64_t)bh * 64 * lpad_g;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;

    // stage K (rows >= L zero) and V^T (16-byte chunks; columns >= L zeroed below)
    for (int c = tid; c < LP * 8; c += 256) {
        const int r = c >> 3, kc = c & 7;
        uint4 v = make_uint4(0, 0, 0, 0);
        if (r < L) v = *(const uint4*)(kh + (int64_t)r * 64 + kc * 8);
        *(uint4*)(sK + kswz(r, kc)) = v;
    }
    const int vchunks = LP / 8;
    for (int c = tid; c < 64 * vchunks; c += 256) {
        const int d = c / vchunks, kc = c % vchunks;
        uint4 v = make_uint4(0, 0, 0, 0);
        if (kc * 8 < lpad_g) v = *(const uint4*)(vh + (int64_t)d * lpad_g + kc * 8);
        *(uint4*)(sV + d * vstride + kc * 8) = v;
    }
    __syncthreads();
    for (int c = tid; c < 64 * (LP - L); c += 256) {
        const int d = c / (LP - L), t = L + c % (LP - L);
        sV[d * vstride + t] = (__bf16)0.0f;
    }
    __syncthreads();

    const int nqb = (L + 15) / 16;
    const int g = lane >> 4, ql = lane & 15;
    for (int qb = wid; qb < nqb; qb += 4) {
        const int qi = qb * 16 + ql;  // this lane's query row
        bf16x8 qf0, qf1;
        if (qi < L) {
            qf0 = *(const bf16x8*)(qh + (int64_t)qi * 64 + g * 8);
            qf1 = *(const bf16x8*)(qh + (int64_t)qi * 64 + 32 + g * 8);
        } else {
            qf0 = bf16x8{};
            qf1 = bf16x8{};
        }
        f32x4 s[NKB];
#pragma unroll
        for (int kb = 0; kb < NKB; kb++) {
            const int kr = kb * 16 + ql;
            const bf16x8 k0 = *(const bf16x8*)(sK + kswz(kr, g));
            const bf16x8 k1 = *(const bf16x8*)(sK + kswz(kr, 4 + g));
            f32x4 a = f32x4{0.f, 0.f, 0.f, 0.f};
            a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(k0, qf0, a, 0, 0, 0);
            a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(k1, qf1, a, 0, 0, 0);
            s[kb] = a;  // s[kb][r] = S[query qi][key kb*16 + 4g + r]
        }
        // masked row max
        float mx = -__builtin_inff();
#pragma unroll
        for (int kb = 0; kb < NKB; kb++)
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int key = kb * 16 + 4 * g + r;
                const bool ok = key < L && (!CAUSAL || key <= qi);
                s[kb][r] = ok ? s[kb][r] : -__builtin_inff();
                mx = fmaxf(mx, s[kb][r]);
            }
        mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
        const float mb = mx * scale_log2;
        float sum = 0.f;
#pragma unroll
        for (int kb = 0; kb < NKB; kb++)
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const float p = exp2f(s[kb][r] * scale_log2 - mb);
                s[kb][r] = p;
                sum += p;
            }
        sum += __shfl_xor(sum, 16, 64);
        sum += __shfl_xor(sum, 32, 64);
        const float inv = 1.0f / sum;
        // O^T[d][q] = sum_key V^T[d][key] P^T[key][q]; k-slot 8g+t <-> key 32s+4g+t (t<4),
        // 32s+16+4g+(t-4) (t>=4) on both operands.
        f32x4 oacc[4];
#pragma unroll
        for (int db = 0; db < 4; db++) oacc[db] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int st = 0; st < NKB / 2; st++) {
            bf16x8 pf;
#pragma unroll
            for (int t = 0; t < 4; t++) {
                pf[t] = (__bf16)s[2 * st][t];
                pf[4 + t] = (__bf16)s[2 * st + 1][t];
            }
#pragma unroll
            for (int db = 0; db < 4; db++) {
                const __bf16* vr = sV + (db * 16 + ql) * vstride + 32 * st + 4 * g;
                const bf16x4 v0 = *(const bf16x4*)(vr);
                const bf16x4 v1 = *(const bf16x4*)(vr + 16);
                const bf16x8 vf = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
                oacc[db] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf, oacc[db], 0, 0, 0);
            }
        }
        if (qi < L) {
            __bf16* orow = o + ((int64_t)b * L + qi) * (H * 64) + h * 64;
#pragma unroll
            for (int db = 0; db < 4; db++) {
                bf16x4 w = {(__bf16)(oacc[db][0] * inv), (__bf16)(oacc[db][1] * inv), (__bf16)(oacc[db][2] * inv),
                            (__bf16)(oacc[db][3] * inv)};
                *(bf16x4*)(orow + db * 16 + 4 * g) = w;
            }
        }
    }
}

// V^T LDS row stride (elements): >= LP and == 4 dwords mod 64 dwords, so the 16 rows x 2
// lane groups of one ds_read_b64 land on distinct banks.
static int vt_stride(int lp) {
    int dw = lp / 2;
    int pad = ((4 - dw) % 64 + 64) % 64;
    return (dw + pad) * 2;
}

template <int NKB, bool CAUSAL>
static int launch_mhsa(const void* q, const void* k, const void* vt, void* o, int64_t nseq, int L, int H,
                       int lpad_g, hipStream_t s) {
    constexpr int LP = NKB * 16;
    const int vs = vt_stride(LP);
    const size_t lds = (size_t)LP * 64 * 2 + (size_t)64 * vs * 2;
    const float scale_log2 = 0.125f * 1.4426950408889634f;  // 1/sqrt(64) * log2(e)
    if (lds > 64 * 1024)
        RM_CHECK_HIP(hipFuncSetAttribute((const void*)mhsa_kernel<NKB, CAUSAL>,
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL((mhsa_kernel<NKB, CAUSAL>), dim3((unsigned)(nseq * H)), dim3(256), lds, s,
                       (const __bf16*)q, (const __bf16*)k, (const __bf16*)vt, (__bf16*)o, L, H, lpad_g, vs,
                       scale_log2);
    RM_LAUNCHED();
    return OK;
}

// Smallest instantiated key-padding >= L.  Lp must also equal the vt row length the
// QKV epilogue wrote (attn_lpad()).
int attn_lpad(int L) {
    if (L <= 96) return 96;
    if (L <= 128) return 128;
    if (L <= 224) return 224;
    if (L <= 256) return 256;
    return -1;
}

int mhsa(const void* q, const void* k, const void* vt, void* o, int64_t nseq, int L, int H, bool causal,
         hipStream_t s) {
    const int lp = attn_lpad(L);
    RM_REQUIRE(lp > 0, "mhsa: sequence length must be <= 256");
    RM_REQUIRE(nseq * H < (1ll << 31), "mhsa: too many (sequence, head) pairs");
    if (causal) {
        switch (lp) {
            case 96: return launch_mhsa<6, true>(q, k, vt, o, nseq, L, H, lp, s);
            case 128: return launch_mhsa<8, true>(q, k, vt, o, nseq, L, H, lp, s);
            case 224: return launch_mhsa<14, true>(q, k, vt, o, nseq, L, H, lp, s);
            default: return launch_mhsa<16, true>(q, k, vt, o, nseq, L, H, lp, s);
        }
    }
    switch (lp) {
        case 96: return launch_mhsa<6, false>(q, k, vt, o, nseq, L, H, lp, s);
        case 128: return launch_mhsa<8, false>(q, k, vt, o, nseq, L, H, lp, s);
        case 224: return launch_mhsa<14, false>(q, k, vt, o, nseq, L, H, lp, s);
        default: return launch_mhsa<16, false>(q, k, vt, o, nseq, L, H, lp, s);
    }
}

}  // namespace reidmi

using namespace reidmi;

REIDMI_API int reidmi_attn_lpad(int L) { return attn_lpad(L); }

REIDMI_API int reidmi_mhsa_bf16(const void* q, const void* k, const void* vt, void* o, int64_t nseq, int L, int H,
                                int causal, void* stream) {
    return mhsa(q, k, vt, o, nseq, L, H, causal != 0, (hipStream_t)stream);
}
