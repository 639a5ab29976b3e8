/*
 * reidmi_tools.h — entry points of libreidmi_tools.so only: the product library
 * (libreidmi.so, reidmi.h) plus the forced-variant calls that tests and A/B tools use to
 * check that every kernel choice gives the same bits and to time one choice against another.
 * None of them is on the product path: the product library is built without them
 * (REIDMI_TOOLS undefined), and multimodal_reid_amd._lib.load_tools() loads this one.
 */
#ifndef REIDMI_TOOLS_H
#define REIDMI_TOOLS_H
#include "reidmi.h"

#ifdef __cplusplus
extern "C" {
#endif

/* reidmi_distmat_f32 with an explicit kernel choice (no process-global state): variant 0 =
 * auto (K-step-32 pipelined kernel when D, ldq, ldg are multiples of 4 and the operands 16-byte
 * aligned), 1 = single-stage kernel.  Both run the same MFMA sequence per output: bit-identical. */
int reidmi_distmat_f32_variant(const float* q, int64_t Q, int64_t ldq, const float* g, int64_t G, int64_t ldg,
                               int64_t D, float* out, int64_t ldo, float* ws, int variant, void* stream);

/* reidmi_gemm_f16 with an explicit tiling: tile 0 = auto (the persistent 256x256x64 LDS-DMA
 * tile for >= 256 tiles, else 128x128x64), 1 = force 128x128, 2 = force persistent; ngroups =
 * the persistent walk's XCD groups (1, 2, 4, 8; each owns 1/ngroups of the N-tiles), 0 = auto.
 * Every choice is bit-identical. */
int reidmi_gemm_f16_tiled(int epi, const void* A, int64_t lda, const void* W, int64_t ldw, int64_t M, int64_t N,
                          int64_t K, const float* bias, const void* rowstat, const float* colsum, void* out,
                          int64_t ldc, int tile, int ngroups, void* stream);

/* ln_1 -> in_proj -> SDPA of one encoder block (custom_clip_model.py:22-27) with ln_1 folded
 * (reidmi_gemm_f16's rowstat / colsum / folded bias; wq [3W][ldw] = the folded in_proj weight):
 * o [nseq*L][W] fp16 = attention output, token-major.  fused = 1: one kernel, q / k / v stay on
 * chip (192 < L <= 224, non-causal; q, k, vt may be NULL); fused = 0: the QKV GEMM into q, k
 * [nseq*H][L][64] and vt [nseq*H][64][reidmi_attn_lpad(L)] then reidmi_mhsa_f16 — what
 * reidmi_vit_forward runs (the fused kernel is bit-identical but measured slower). */
int reidmi_qkv_attention_f16(const void* x, int64_t ldx, const void* wq, int64_t ldw, const float* bias,
                             const float* colsum, const void* rowstat, int64_t nseq, int L, int H, int W, void* q,
                             void* k, void* vt, void* o, int fused, void* stream);

/* The QKV GEMM alone (ln_1 fold + the head split reidmi_vit_forward uses): x [nseq*L][lda],
 * W [3*H*64][ldw] -> q, k [nseq*H][L][64], vt [nseq*H][64][lpad] (lpad = reidmi_attn_lpad(L)). */
/* One-wave-per-SIMD GEMM prototype (gemm.hip gemm_w4_kernel): out fp16 = A.W^T + bias, same MFMA
 * chain as reidmi_gemm_f16 epi 0 (bit-identical); nostore: the values are computed, not stored.
 * N % 256 == 0, K % 64 == 0, K >= 128. */
int reidmi_gemm_f16_w4(const void* A, int64_t lda, const void* W, int64_t ldw, int64_t M, int64_t N, int64_t K,
                       const float* bias, void* out, int64_t ldc, int nostore, void* stream);

/* The round-robin vision attention kernel (mhsa_rr_kernel: 8 waves walk (head, 32-query block)
 * units over three LDS slots) for non-causal 205 <= L <= 212 with V^T rows of 212 elements:
 * bit-identical to reidmi_mhsa_f16 (which takes V^T rows of reidmi_attn_lpad(L)), measured no
 * faster, so only the tools library has it. */
int reidmi_mhsa_f16_rr(const void* q, const void* k, const void* vt, void* o, int64_t nseq, int L, int H,
                       void* stream);

int reidmi_gemm_f16_qkv(const void* A, int64_t lda, const void* W, int64_t ldw, int64_t nseq, int L, int H,
                        const float* bias, const void* rowstat, const float* colsum, void* q, void* k, void* vt,
                        int lpad, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* REIDMI_TOOLS_H */
