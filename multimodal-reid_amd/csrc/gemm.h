// gemm.h — fp16 MFMA GEMM with fused epilogues for the CLIP encoders (gfx950).
//
// C[M,N] = A[M,K] . W[N,K]^T (+ bias[N]), A row-major fp16 (activations), W row-major fp16
// (PyTorch Linear / conv weight layout [out, in]), fp32 accumulation on
// v_mfma_f32_16x16x32_f16 (the reference's own GPU dtype, utils.py:145-166).  Epilogues
// implement the ops that follow each GEMM in custom_clip_model.py:8-29 / maple.py:617-644
// so no elementwise pass touches HBM:
//   EPI_H16       out fp16 = acc + bias                       (generic)
//   EPI_GELU_H16  out fp16 = QuickGELU(acc + bias)            (mlp.c_fc + gelu, :14-16,52-54)
//   EPI_QKV       q,k -> [B,H,L,64] fp16, v -> [B,H,64,Lp]    (attn.in_proj + head split)
//   EPI_PATCH     x[b*L+1+p] = acc + pos[1+p]  fp16           (conv1 + pos-embed, :78-86)
//   EPI_F32       out fp32 = acc + bias                       (proj / text_projection), or with
//                 dist_rsq the Euclidean distance (rsq_m + csq_n) - 2 acc (distlowp.hip)
//   EPI_RESID_F16 x fp16 += acc + bias (fp32 sum, one rounding) (out_proj / c_proj + residual, :27-28)
//   EPI_RRHI      out fp32 = hi(i, j), the upper bound of the exact distance of items i, j from their
//                 fp16 product (the k-reciprocal re-rank's pre-filter, rerank.hip): only the bound
//                 reaches HBM, and the selection reads 4 bytes per pair instead of 12
//   EPI_RRSV      no dense output: the pairs of row i that can still matter to its R2 selection
//                 (hi <= hi_max_i or hi >= lb_i, per-row thresholds from a sampled pass) are
//                 appended to the row's survivor list, ~1 000 of the N columns (persistent tile
//                 only; with rr_tri the upper triangle of a symmetric product, each pair tested
//                 for both its rows)
#pragma once
#include "common.h"

namespace reidmi {

enum Epi : int {
    EPI_H16 = 0,
    EPI_GELU_H16 = 1,
    EPI_QKV = 3,
    EPI_PATCH = 4,
    EPI_F32 = 5,
    EPI_RESID_F16 = 6,
    EPI_RRHI = 7,
    EPI_RRSV = 8
};

struct EpiArgs {
    void* out;          // fp16 / fp32 output (or residual x for RESID, x for PATCH)
    int64_t ldc;        // row stride of out (elements)
    const float* bias;  // [N] or null
    // QKV head split
    void* q;
    void* k;
    void* vt;
    int seq;    // L (tokens per sequence)
    int heads;  // H
    int lpad;   // Lp (row length of vt)
    int n_off;  // QKV: column offset of this GEMM inside [q | k | v] (a GEMM may produce k,v only)
    // PATCH
    const float* pos;  // [1+NP][N]
    int npatch;        // NP
    // LayerNorm folded into the GEMM: with W' = W diag(gamma) (fp16),
    // s_n = sum_k W'[n,k], b' = b + W beta (the bias above):
    //   LN(x) W^T + b = rstd_m * (x W'^T)_mn + (-mean_m rstd_m) * s_n + b'_n
    const float2* rowstat;  // [round_up(M, 256)] (rstd, -mean*rstd) of the A rows (entries
                            // past M are read, not used), or null (no fold)
    const float* colsum;    // [N] s_n
    // EPI_RESID_F16: LayerNorm partials of the updated rows, or null.  pstat[c * ldp + m]
    // = (sum, sum of (v - sum/64)^2) of row m over columns [64c, 64c + 64) of the fp16
    // values written (column-block-major, ldp >= M: 16 consecutive rows per store and
    // coalesced reads in the encoder's rowstat_combine_kernel)
    float2* pstat;
    int64_t ldp;
    // EPI_RRHI: row m is item rr_row0 + m, column n item n (n >= rr_n: +inf); squared norms and
    // norms of the items; the bound's constants (c_rel, c_abs, c_d: backend.hip rank_select)
    const float* rr_sqn;
    const float* rr_nrm;
    int64_t rr_row0;
    int64_t rr_n;
    float rr_c[3];
    const float* rr_csqn;  // the columns' squared norms / norms when they are not items 0..rr_n-1
    const float* rr_cnrm;  // (a sampled item set); null: rr_sqn / rr_nrm
    // EPI_RRSV: per row m the record rr_rowmeta[m] = (s_m, n_m, hi_max, lb) -- a pair with
    // hi <= hi_max can be a candidate of the K smallest, a pair with hi >= lb can hold the row's
    // largest distance -- padded to whole 256-row tiles; per column c < Np the record
    // rr_colrec[c] = (s_c, n_c, hi_max, lb) (thresholds used with rr_tri only); the survivor
    // counters and lists [m * sv_cap + p] = (column, hi bits) of the pairs with
    // !(hi_max < hi < lb) (a NaN survives); counts past sv_cap are kept (the row then takes the
    // exact path).  rr_tiles (optional): the tiles to run, (M-tile << 16 | N-tile), rr_ntiles
    // of them; rr_tri: rows and columns are the same items (A = W), the list holds tiles with
    // M-tile <= N-tile, and a tile above the diagonal also tests each pair as (column, row)
    // against the column item's thresholds (its row of the symmetric product)
    const float4* rr_rowmeta;
    const float4* rr_colrec;
    const int* rr_tiles;
    int64_t rr_ntiles;
    int rr_tri;
    int* sv_cnt;
    int2* sv_list;
    int sv_cap;
    // EPI_F32 distance form (dist_rsq non-null): out[m][n] = (dist_rsq[m] + dist_csq[n]) - 2 acc
    // for n < dist_n (columns past it are not written; out may be any fp32 row pitch >= dist_n)
    const float* dist_rsq;
    const float* dist_csq;
    int64_t dist_n;
};

// hi(i, j) = fl(dt + e), dt = fl(fma(-2, dot, s_i + s_j)),
// e = 1.01 (fma(c_rel n_i, n_j, 2^-23 (s_i + s_j)) + c_abs (n_i + n_j) + c_d): the exact fp32
// distance of i and j is <= hi and >= fl(dt - e) (backend.hip rank_select).  One definition for
// the GEMM epilogue and the selection's re-evaluation of single pairs.
__device__ __forceinline__ float rr_hi(float dot, float si, float sj, float crn_i, float ni, float nj,
                                       const float (&c)[3]) {
    const float s = si + sj;
    const float dt = __builtin_fmaf(-2.0f, dot, s);
    const float e = 1.01f * (__builtin_fmaf(crn_i, nj, 0x1p-23f * s) + c[1] * (ni + nj) + c[2]);
    return dt + e;
}

// Per-call tiling choice (tests, A/B tools): tile 0 = auto (the persistent 256x256 LDS-DMA
// tile when the GEMM has >= 256 of them, else 128x128), 1 = force 128x128, 2 = force
// persistent; ngroups = XCD N-groups of the persistent walk (0 = auto, 1, 2, 4, 8).  Every
// choice runs the same MFMA chain per output element: bit-identical results.
struct GemmOpts {
    int tile = 0;
    int ngroups = 0;
    int band = -1;  // persistent walk: M-tiles per band (0 = M-major, -1 = auto; gemm.hip tile_mn)
};

// Launch C = A . W^T with epilogue `epi`.  Requires N % 128 == 0, K % 64 == 0, lda/ldw
// multiples of 8 (16-byte rows); M arbitrary.  ea.rowstat / ea.colsum enable the fold.
int gemm_f16(int epi, const void* A, int64_t lda, const void* W, int64_t ldw, int64_t M, int64_t N, int64_t K,
             const EpiArgs& ea, hipStream_t stream, const GemmOpts& opts = GemmOpts{});

}  // namespace reidmi
