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

namespace reidmi {

int attn_lpad(int L);

__device__ __forceinline__ int kswz(int r, int kc) { return r * 64 + ((kc ^ ((r >> 1) & 7)) << 3); }

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef float f32x2v __attribute__((ext_vector_type(2)));

// One wave's block of 32 queries (row qi = block * 32 + (lane & 31)) against the head's K
// [LP][64] and V^T [64][vstride] in LDS:
//   S^T[key][q] = K Q^T on v_mfma_f32_32x32x16_f16; lane (q = lane&31, h = lane>>5) holds
//     keys kb*32 + (r&3) + 8(r>>2) + 4h in s[kb][r];
//   P stays in registers: registers 8s'..8s'+7 of block kb are the B fragment of key-step s'
//     of O^T = V^T P^T (accumulator-as-operand), V^T read with the same key permutation;
//   O^T[d][q] comes out as 4 runs of 4 consecutive d per lane -> 8 8-byte stores (the wave's
//     only vector-memory ops here; lanes with qi >= L store nothing).
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
#pragma unroll
        for (int db = 0; db < 2; db++)
#pragma unroll
            for (int g = 0; g < 4; g++) {
                f16x4 w = {(_Float16)(oacc[db][4 * g] * inv), (_Float16)(oacc[db][4 * g + 1] * inv),
                            (_Float16)(oacc[db][4 * g + 2] * inv), (_Float16)(oacc[db][4 * g + 3] * inv)};
                *(f16x4*)(orow + db * 32 + 8 * g + 4 * hh) = w;
            }
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

template <int NKB, bool CAUSAL>
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
            asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)" ::: "memory");
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

// V^T row stride (elements): LP + 4, i.e. LP/2 + 2 dwords, which is 2 mod 4 dwords (LP is a
// multiple of 32): the 32 rows of one half-wave ds_read_b64 then start on 32 distinct even
// banks (row r at bank 2 * (r * odd mod 32)), so they cover all 64 banks exactly once.  (The
// stride 2 mod 64 used before padded V^T by up to 60 elements per row: 23 % of V at L = 211.)
// The QKV epilogue writes V^T with this same stride in HBM, so one head's V^T is a contiguous
// blob for the LDS-DMA copy; 64 * (LP + 4) * 2 bytes is a multiple of 512.
static int vt_stride(int lp) { return lp + 4; }

static int g_num_cu = 0;
static int num_cu() {
    if (!g_num_cu) {
        int dev = 0;
        hipGetDevice(&dev);
        hipDeviceGetAttribute(&g_num_cu, hipDeviceAttributeMultiprocessorCount, dev);
        if (g_num_cu <= 0) g_num_cu = 256;
    }
    return g_num_cu;
}

template <int NKB, bool CAUSAL>
static int launch_mhsa(const void* q, const void* k, const void* vt, void* o, int64_t nseq, int L, int H,
                       int lpad_g, hipStream_t s) {
    constexpr int LP = NKB * 32;
    const int vs = vt_stride(LP);
    RM_REQUIRE(lpad_g == vs, "mhsa: v^T row stride must be reidmi_attn_lpad(L)");
    const size_t stage = (size_t)LP * 64 * 2 + (size_t)64 * vs * 2;
    const size_t lds = 2 * stage;
    const float scale_log2 = 0.125f * 1.4426950408889634f;  // 1/sqrt(64) * log2(e)
    static bool attr = false;
    if (!attr) {
        RM_CHECK_HIP(hipFuncSetAttribute((const void*)mhsa_kernel<NKB, CAUSAL>,
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
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
        RM_CHECK_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, (const void*)mhsa_kernel<NKB, CAUSAL>,
                                                                  64 * waves, lds));
        occ = n > 0 ? n : 1;
        occ_waves = waves;
    }
    const int64_t slots = (int64_t)num_cu() * occ;
    const int64_t grid = nbh < slots ? nbh : slots;
    hipLaunchKernelGGL((mhsa_kernel<NKB, CAUSAL>), dim3((unsigned)grid), dim3(64 * waves), lds, s,
                       (const _Float16*)q, (const _Float16*)k, (const _Float16*)vt, (_Float16*)o, L, H, vs, nbh,
                       scale_log2);
    RM_LAUNCHED();
    return OK;
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

REIDMI_API int reidmi_mhsa_f16(const void* q, const void* k, const void* vt, void* o, int64_t nseq, int L, int H,
                                int causal, void* stream) {
    return mhsa(q, k, vt, o, nseq, L, H, causal != 0, (hipStream_t)stream);
}
