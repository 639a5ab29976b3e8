/*
 * reidmi.h — C ABI of libreidmi.so, the MI355X-native CLIP-ReID inference +
 * retrieval path.  Plain pointers and sizes only: every pointer argument is a
 * device pointer (caller-owned, e.g. torch tensor .data_ptr()) unless noted; every
 * call is stream-ordered on `stream` (a hipStream_t passed as void*) and never
 * allocates or synchronises, so a caller may capture it into a hipGraph.
 * Return value: 0 on success, non-zero status with reidmi_last_error() set.
 *
 * The reference (SuperbTUM/Multimodal-ReID) is pure Python with no FFI; each entry
 * point below names the reference function whose semantics it implements.  The
 * Python binding (ctypes) that re-exports the reference call surface lives in
 * multimodal-reid_amd/_lib.py; INTEGRATION.md shows how a reference checkout
 * would bind it.
 */
#ifndef REIDMI_H
#define REIDMI_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define REIDMI_OK 0
#define REIDMI_EINVAL 1
#define REIDMI_EHIP 2
#define REIDMI_ECAP 3

const char* reidmi_last_error(void);
/* 4 since round 4: the A/B-only entry points (forced GEMM tiling, distance-kernel variant, the
 * fused QKV + attention kernel) moved to the tools library (include/reidmi_tools.h). */
int reidmi_abi_version(void);

/* ------------------------------------------------------------ retrieval back end */

/* sum_k x[i,k]^2 as an fmaf chain over k ascending (building block of the two below). */
int reidmi_row_sqnorm_f32(const float* x, int64_t n, int64_t d, int64_t ldx, float* out, void* stream);

/* torch.nn.functional.normalize(feats, dim=1, p=2)  — evaluate.py:114.
 * ws: n floats. */
int reidmi_l2norm_f32(const float* x, int64_t n, int64_t d, int64_t ldx, float* y, int64_t ldy, float* ws,
                      void* stream);

/* euclidean_distance(qf, gf) — evaluate.py:7-13 (also reranking.py:36-41 with q = g = feat).
 * out[i*ldo+j] = (||q_i||^2 + ||g_j||^2) - 2 q_i.g_j in exact fp32 (v_mfma_f32_32x32x2_f32).
 * ws: Q+G floats. */
int reidmi_distmat_f32(const float* q, int64_t Q, int64_t ldq, const float* g, int64_t G, int64_t ldg, int64_t D,
                       float* out, int64_t ldo, float* ws, void* stream);

/* Reduced-precision mode of euclidean_distance (SURVEY.md §8b "reidmi_distmat ... mode"):
 * out[i*ldo+j] = (||q_i||^2 + ||g_j||^2) - 2 fp16(q_i).fp16(g_j), the dot products on the fp16
 * MFMA GEMM (fp32 accumulation), the squared norms exact fp32.  Not bit-exact with the
 * reference (reidmi_distmat_f32 is); |error| <= 2^-8 ||q_i|| ||g_j|| per entry (fp16-range rows).
 * The GEMM's epilogue writes the distances straight into out (no product buffer).
 * ws: reidmi_distmat_f16_workspace_bytes(Q, G, D) bytes (fp16 copies padded to the GEMM tile,
 * the squared norms). */
int64_t reidmi_distmat_f16_workspace_bytes(int64_t Q, int64_t G, int64_t D);
int reidmi_distmat_f16(const float* q, int64_t Q, int64_t ldq, const float* g, int64_t G, int64_t ldg, int64_t D,
                       float* out, int64_t ldo, void* ws, int64_t ws_bytes, void* stream);

/* cosine_similarity(qf, gf) — evaluate.py:16-26: arccos(clip(q.g / (|q||g|), -1+1e-5, 1-1e-5)).
 * Same tiling as reidmi_distmat_f32; ws: Q+G floats. */
int reidmi_cosine_f32(const float* q, int64_t Q, int64_t ldq, const float* g, int64_t G, int64_t ldg, int64_t D,
                      float* out, int64_t ldo, float* ws, void* stream);

/* np.argsort(x, axis=1)[:, :k] with ties in index order (kind="stable") — evaluate.py:40,
 * reranking.py:48.  row_div (nullable): rows are divided by row_div[row] first
 * (reranking.py:46 column-max normalisation of a symmetric distance).  Any k <= cols (k > 1024
 * runs in rounds of 1024, one stream over the row each).
 * out_val (nullable) receives the selected values. */
int reidmi_topk_rows_f32(const float* x, int64_t rows, int64_t cols, int64_t ldx, const float* row_div, int k,
                         int32_t* out_idx, float* out_val, int64_t ldo, void* stream);

/* Per-query part of eval_func — evaluate.py:40-80.  For query q: valid[q] (any match kept),
 * first[q] (0-based kept-rank of the first match), ap[q] (float64 AP exactly as numpy sums
 * it), nkept[q] (gallery items left after same-pid-same-cam removal).  No capacity limit
 * on positives or junk items per query.  overflow: one int32, written 0 by the call (kept for
 * ABI compatibility with builds that had a positive-list capacity). */
int reidmi_eval_rows(const float* dist, int64_t Q, int64_t G, int64_t ldd, const int64_t* q_pids,
                     const int64_t* g_pids, const int64_t* q_cams, const int64_t* g_cams, int32_t* valid,
                     int64_t* first, double* ap, int64_t* nkept, int32_t* overflow, void* ws, int64_t ws_bytes,
                     void* stream);
/* Device workspace bytes (16-byte aligned) for reidmi_eval_rows: the gallery labels packed
 * once per call and the scratch of a query with more positives than fit LDS (O(G)). */
int64_t reidmi_eval_rows_workspace_bytes(int64_t G);


/* k-reciprocal re-ranking — re_ranking(probFea, galFea, k1, k2, lambda_value) (reranking.py:29-100),
 * bit-exact with the reference's numpy arithmetic given the same distances (stable ties).
 * feat [Q+G][ldf] fp32 = cat(probFea, galFea).  final_dist [Q][ldo] fp32 = re-ranked q x g
 * distances.  one_minus_lambda_h = np.float16(1 - lambda) bits, lambda_f = np.float32(lambda)
 * (numpy's weak-scalar conversions, reranking.py:95).  Any k1 >= 1, k2 >= 1 and any neighbourhood
 * density (no capacity limit, as the reference): the workspace holds V and V_qe at their
 * worst-case row widths (kf (kh1 + 1) and k2 times that, capped at N) and the scratch of the
 * kernels for rows beyond the on-chip ones.  flags: device int32, 0 after a correct run (8 would
 * mean a row beyond the sized scratch: a bug, reported instead of a fault). */
int64_t reidmi_rerank_workspace_bytes(int64_t Q, int64_t G, int k1, int k2, int from_dist, int need_transpose);
int reidmi_rerank(const float* feat, int64_t Q, int64_t G, int64_t D, int64_t ldf, int k1, int k2,
                  uint16_t one_minus_lambda_h, float lambda_f, float* final_dist, int64_t ldo, void* ws,
                  int64_t ws_bytes, int32_t* flags, void* stream);
/* From a given (Q+G) x (Q+G) distance (reranking.py:33-35 only_local / local_distmat paths):
 * original_dist = dist (+ add, nullable); symmetric = 1 promises original_dist == its
 * transpose (then no transpose pass is made). */
int reidmi_rerank_from_dist(const float* dist, const float* add, int64_t Q, int64_t G, int symmetric, int k1,
                            int k2, uint16_t one_minus_lambda_h, float lambda_f, float* final_dist, int64_t ldo,
                            void* ws, int64_t ws_bytes, int32_t* flags, void* stream);

/* Staged re-ranking: R1-R7 of re_ranking (reranking.py:29-100) as row-range stages over
 * caller-allocated, exactly sized buffers, bit-identical to reidmi_rerank.  The N x N distance
 * is never materialised (chunk_rows x N row blocks are), and every stage takes a row range,
 * so ranks can each own [lo, hi) and all-gather R / V / V_qe between stages.
 * feat [N][ldf] fp32 = cat(probFea, galFea); sqn[N] = squared row norms (reidmi_row_sqnorm_f32).
 * K = min(max(k1 + 1, k2), N) columns of initial_rank.  CSR inputs are (off[N+1] int64, col
 * int32, fp16 bits), columns ascending per row.
 * reidmi_rr_caps: ELL widths vcap (V rows: the bound kf (kh1 + 1), capped at N) and qcap (the
 * V_qe rows reidmi_rr_qe_rows assembles on chip), and the workspace bytes of reidmi_rr_v_rows
 * (0 when k1 <= 61: on chip) and of reidmi_rr_qe_deferred. */
int reidmi_rr_caps(int64_t N, int k1, int k2, int64_t* vcap, int64_t* qcap, int64_t* v_ws_bytes,
                   int64_t* qe_ws_bytes);
/* R1+R2 (reranking.py:36-48): rank_out[hi-lo][K] = stable argsort prefix of od rows lo..hi,
 * rowmax_out[hi-lo] = the od divisors (column maxima of the symmetric distance). */
int reidmi_rr_rank_rows(const float* feat, int64_t N, int64_t D, int64_t ldf, const float* sqn, int64_t lo, int64_t hi,
                        int K, int32_t* rank_out, float* rowmax_out, float* chunk, int64_t chunk_rows, void* stream);
/* R3 (reranking.py:51-71): V rows lo..hi (ELL [hi-lo][vcap]) from the full rank[N][K] and
 * rowmax[N]; distance entries recomputed from feat with the distance kernel's arithmetic. */
/* fp16 copy of the features for reidmi_rr_rank_rows_f16: [Np][Dp] zero-padded (Np % 256 == 0,
 * Dp % 64 == 0); *range_ok (device int32, set to 1 by the caller) is cleared when some |x| > 2^15
 * or is not finite, and the pre-filter must then not be used. */
int reidmi_rr_feat16(const float* feat, int64_t N, int64_t D, int64_t ldf, void* feat16, int64_t Np, int64_t Dp,
                     int32_t* range_ok, void* stream);
/* Largest norm and squared norm over the N items (out2[0], out2[1]: device floats), the input
 * nmax2 of reidmi_rr_rank_rows_f16. */
int reidmi_rr_norm_max(const float* sqn, const float* nrm, int64_t N, float* out2, void* stream);
/* reidmi_rr_rank_rows with an fp16 MFMA pre-filter (same rank_out / rowmax_out bits): the fp16
 * product bounds every exact distance (error bound in backend.hip rank_select_kernel); only the
 * candidates are recomputed with the exact fp32 chain.  Default form (sample stride 16, for N
 * >= 4096): per-row thresholds from every 16th item, then the selection runs inside the GEMM's
 * epilogue (survivor lists, no N-wide row in HBM; when one call covers all N rows and the lists
 * fit the chunk, only the upper triangle of the symmetric product runs).  Smaller N: the GEMM's
 * epilogue writes the upper bounds (chunk [chunk_rows][Np] fp32) for a streaming selection.
 * Rows whose distances are too concentrated for the bound (or not finite), or whose survivor
 * list overflows, get need[r] = 1 and no output: the caller runs the exact rows for them.
 * nrm = sqrt(sqn); nmax2 = reidmi_rr_norm_max(sqn, nrm); need [hi - lo] int32; chunk:
 * chunk_rows x Np fp32. */
int reidmi_rr_rank_rows_f16(const float* feat, int64_t N, int64_t D, int64_t ldf, const float* sqn, const float* nrm,
                            const float* nmax2, const void* feat16, int64_t Np, int64_t Dp, int64_t lo, int64_t hi,
                            int K, int32_t* rank_out, float* rowmax_out, int32_t* need, float* chunk,
                            int64_t chunk_rows, void* stream);
/* The same with the sample stride chosen: 0 or 1 = the dense form (bounds written to the chunk,
 * streaming selection) at any N; S >= 2 = the selection inside the GEMM's epilogue against
 * per-row thresholds from every S-th item (backend.hip "R2 pre-filter with the selection in the
 * GEMM"), when floor(N / S) spans at least one 256-column tile and 4 K items (else the dense
 * form).  Same output bits.  reidmi_rr_rank_rows_f16 uses S = 16 (rerank.hip RR_SAMPLE_STRIDE):
 * 1M-item R2 1.98 s in the triangle form vs 3.9 s dense. */
int reidmi_rr_rank_rows_f16_ex(const float* feat, int64_t N, int64_t D, int64_t ldf, const float* sqn,
                               const float* nrm, const float* nmax2, const void* feat16, int64_t Np, int64_t Dp,
                               int64_t lo, int64_t hi, int K, int32_t* rank_out, float* rowmax_out, int32_t* need,
                               float* chunk, int64_t chunk_rows, int sample_stride, void* stream);
/* Rows that one internal pass of reidmi_rr_rank_rows_f16(_ex) processes with a chunk of
 * chunk_rows x Np floats (the in-epilogue form needs ~0.3 MB per row at N = 1M instead of 4 N
 * bytes): size the calls' row ranges by it.  sample_stride < 0: the default form's.  -1 on bad
 * arguments. */
int64_t reidmi_rr_rank_rows_f16_pass_rows(int64_t N, int64_t Np, int64_t chunk_rows, int K, int sample_stride);
/* R2's triangle form in stages, for sharding it over ranks (reranking.HipStages under a process
 * group): rank r samples its rows (reidmi_rr_tri_sample, records all-gathered), runs tiles
 * [t0, t1) = its contiguous share of the upper-triangle list over ALL rows
 * (reidmi_rr_tri_survivors), sends the partial survivor lists of each other rank's rows to it
 * (reidmi_rr_sv_pack, all-to-all) which appends them (reidmi_rr_sv_merge), and selects its own
 * rows (reidmi_rr_sv_select): the same rank_out / rowmax_out / need bits as the one-call
 * reidmi_rr_rank_rows_f16 for any number of ranks, at the one-GPU triangle's total MFMA work.
 * Buffers (caller-owned, device): meta [Np] x 16 B, wrow [N] fp32, cnt [N] int32 (0 for rows
 * sampled elsewhere), list [N][cap] x 8 B, sqn_s / nrm_s [ns] fp32, tiles [ntiles] int32, hs
 * [sample_rows][ns] fp32 (may overlay list; the sizes: reidmi_rr_tri_plan; cap = 0: the
 * triangle form does not apply for this chunk). */
int reidmi_rr_tri_plan(int64_t N, int64_t Np, int64_t chunk_rows, int K, int64_t* ntiles, int64_t* cap, int64_t* ns,
                       int64_t* sample_rows);
int reidmi_rr_tri_init(const float* sqn, const float* nrm, int64_t N, int64_t Np, int64_t ns, void* meta, float* sqn_s,
                       float* nrm_s, int32_t* tiles, void* stream);
int reidmi_rr_tri_sample(const void* feat16, int64_t Np, int64_t Dp, const float* sqn, const float* nrm,
                         const float* nmax2, int64_t N, int64_t D, int K, const float* sqn_s, const float* nrm_s,
                         int64_t ns, int64_t a, int64_t b, float* hs, int64_t hs_rows, void* meta, float* wrow,
                         int32_t* cnt, int cap, void* stream);
int reidmi_rr_tri_survivors(const void* feat16, int64_t Np, int64_t Dp, const float* sqn, const float* nrm, int64_t N,
                            int64_t D, const void* meta, const int32_t* tiles, int64_t t0, int64_t t1, int32_t* cnt,
                            void* list, int cap, void* stream);
int reidmi_rr_sv_select(const int32_t* cnt, const void* list, int cap, const float* wrow, const float* feat,
                        int64_t ldf, int64_t D, const float* sqn, int64_t row0, int64_t rows, int K, int32_t* rank_out,
                        float* rowmax_out, int32_t* need, void* stream);
int reidmi_rr_sv_pack(const int32_t* cnt, const void* list, int cap, int64_t rows, const int64_t* off, void* out,
                      void* stream);
int reidmi_rr_sv_merge(int32_t* cnt, void* list, int cap, int64_t rows, const int32_t* add_cnt, const int64_t* add_off,
                       const void* add, void* stream);
/* R3 (reranking.py:51-71): V rows lo..hi (ELL [hi-lo][vcap]) from the full rank[N][K] and
 * rowmax[N]; distance entries recomputed from feat with the distance kernel's arithmetic.
 * ws: reidmi_rr_caps' v_ws_bytes (nullable when 0). */
int reidmi_rr_v_rows(const float* feat, int64_t N, int64_t D, int64_t ldf, const float* sqn, const float* rowmax,
                     const int32_t* rank, int K, int64_t lo, int64_t hi, int k1, int32_t* vcol, uint16_t* vval,
                     int32_t* vnnz, void* ws, int64_t ws_bytes, int32_t* flags, void* stream);
/* off[0..rows] = exclusive scan of nnz[0..rows) (off[rows] = total). */
int reidmi_rr_row_offsets(const int32_t* nnz, int64_t rows, int64_t* off, void* stream);
/* ELL rows -> CSR storage at off[]. */
int reidmi_rr_pack(const int32_t* ell_col, const uint16_t* ell_val, const int32_t* nnz, int64_t rows, int64_t cap,
                   const int64_t* off, int32_t* col, uint16_t* val, void* stream);
/* R4 (reranking.py:73-78): V_qe rows lo..hi (ELL [hi-lo][qcap]) from the full V (CSR).  Rows
 * beyond the on-chip assembly (or every row when k2 > 32) get qnnz = 0 and are listed in
 * dlist[0 .. *dcount) (dlist int32 [hi-lo], dcount device int32, both written by the call);
 * reidmi_rr_qe_deferred then computes them: mode 0 -> their entry counts into qnnz[b], mode 1 ->
 * the rows into CSR at qoff[b] (qoff = offsets of rows lo..hi).  ws: reidmi_rr_caps' qe_ws_bytes. */
int reidmi_rr_qe_rows(const int32_t* rank, int K, int k2, int64_t lo, int64_t hi, const int64_t* voff,
                      const int32_t* vcol, const uint16_t* vval, int32_t* qcol, uint16_t* qval, int32_t* qnnz,
                      int32_t* dlist, int32_t* dcount, void* stream);
int reidmi_rr_qe_deferred(const int32_t* rank, int K, int k1, int k2, int64_t lo, int64_t N, const int64_t* voff,
                          const int32_t* vcol, const uint16_t* vval, const int32_t* dlist, int64_t n_def, int mode,
                          const int64_t* qoff, int32_t* qcol, uint16_t* qval, int32_t* qnnz, void* ws,
                          int64_t ws_bytes, int32_t* flags, void* stream);
/* R5 (reranking.py:80-82): inverted index of the full V_qe (CSR, nnz entries) as CSC with
 * rows ascending per column: coff[N+1], irow[nnz], ival[nnz]. */
int64_t reidmi_rr_csc_workspace_bytes(int64_t N, int64_t nnz);
int reidmi_rr_csc(int64_t N, const int64_t* qoff, const int32_t* qcol, const uint16_t* qval, int64_t nnz, int64_t* coff,
                  int32_t* irow, uint16_t* ival, void* ws, int64_t ws_bytes, void* stream);
/* R6+R7 (reranking.py:84-100): final rows for queries qlo..qhi: out[qhi-qlo][ldo] (G columns).
 * chunk: distance scratch of chunk_rows x G floats (chunk_rows <= 65535); bounds: device
 * scratch of reidmi_rr_jaccard_bounds_bytes(N, G) bytes for the per-column chunk bounds of the
 * inverted lists. */
int reidmi_rr_jaccard_rows(const float* feat, int64_t N, int64_t D, int64_t ldf, const float* sqn,
                           const float* rowmax, int64_t Q, int64_t qlo, int64_t qhi, const int64_t* qoff,
                           const int32_t* qcol, const uint16_t* qval, const int64_t* coff, const int32_t* irow,
                           const uint16_t* ival, uint16_t one_minus_lambda_h, float lambda_f, float* out, int64_t ldo,
                           float* chunk, int64_t chunk_rows, void* bounds, int64_t bounds_bytes, void* stream);
int64_t reidmi_rr_jaccard_bounds_bytes(int64_t N, int64_t G);
/* Row utilities of the staged driver's exact-row fallback (reranking.HipStages): row maxima
 * skipping NaN (the od divisors, reranking.py:46); ordered compaction idx[0..*count) = positions
 * of the nonzero flags (np.nonzero; count: device int32); out[r] = x[row0 + idx[r]] (fp32 rows). */
int reidmi_rowmax_f32(const float* x, int64_t rows, int64_t cols, int64_t ldx, float* out, void* stream);
int reidmi_nonzero_i32(const int32_t* flags, int64_t n, int32_t* idx, int32_t* count, void* stream);
int reidmi_gather_rows_f32(const float* x, int64_t ldx, int64_t d, int64_t row0, const int32_t* idx, int64_t n,
                           float* out, int64_t ldo, void* stream);

/* ---------------------------------------------- multi-GPU exchange (RCCL, §8e) */

/* The eval path's one exchange step for callers that are not Python (the Python drop-in uses
 * torch.distributed's "nccl" group, multimodal_reid_amd/distributed.py, with the same layout):
 * gallery feature rows are sharded contiguously over the ranks of one node — rank r of W owns
 * rows [n*r/W, n*(r+1)/W) — embedded locally, all-gathered (reidmi_comm_allgather_rows), each
 * rank scores its own query rows (reidmi_distmat_f32 + reidmi_eval_rows, or the staged re-rank),
 * and the per-query results are all-gathered the same way and reduced on the host in query
 * order (bit-identical CMC/mAP for every W).  RCCL (NCCL API) is opened at first use from
 * librccl.so.1 (torch's copy when torch is loaded).  No collective is made by any other entry
 * point. */
#define REIDMI_COMM_ID_BYTES 128
typedef struct reidmi_comm* reidmi_comm_t;
/* ncclGetUniqueId: rank 0 creates the id (HOST buffer of REIDMI_COMM_ID_BYTES) and hands it to
 * the other ranks out of band (as for ncclCommInitRank). */
int reidmi_comm_unique_id(void* id);
/* One communicator per process; device = the HIP device of this rank. */
int reidmi_comm_init(reidmi_comm_t* comm, int nranks, int rank, const void* id, int device);
int reidmi_comm_destroy(reidmi_comm_t comm);
int reidmi_comm_rank(reidmi_comm_t comm, int* rank, int* nranks);
/* All-gather of contiguous row shards: send = this rank's rows [n*r/W, n*(r+1)/W) of row_bytes
 * each, recv = all n_total rows in order.  scratch: device, reidmi_comm_allgather_rows_scratch_bytes
 * (W * ceil(n_total / W) * row_bytes; the padded in-place all-gather). */
int64_t reidmi_comm_allgather_rows_scratch_bytes(int nranks, int64_t n_total, int64_t row_bytes);
int reidmi_comm_allgather_rows(reidmi_comm_t comm, const void* send, int64_t n_total, int64_t row_bytes, void* recv,
                               void* scratch, int64_t scratch_bytes, void* stream);
/* Sum all-reduce of count elements; dtype 0 = fp32, 1 = fp64, 2 = int32, 3 = int64. */
int reidmi_comm_allreduce(reidmi_comm_t comm, const void* send, void* recv, int64_t count, int dtype, void* stream);

/* ------------------------------------------------------------------ encoders */

/* fp16 GEMM C = A . W^T (+bias) on v_mfma_f32_16x16x32_f16, fp32 accumulation (the
 * reference's GPU dtype: utils.py:145-166 converts Linear/conv/MHA weights to fp16), with an
 * optional folded LayerNorm — the QKV / c_fc GEMMs of the encoders (ln_1 / ln_2 -> in_proj /
 * c_fc, custom_clip_model.py:27-28):
 * out = epi(rstd_m * (A W^T)_mn + (-mean_m rstd_m) * colsum_n + bias_n), rowstat float2
 * (rstd, -mean * rstd) with round_up(M, 256) entries (those past M are read, not used) and
 * colsum [N] fp32, both NULL for a plain GEMM (bias required with them).
 * A [M][lda], W [N][ldw] fp16 (Linear weight layout), N % 128 == 0, K % 64 == 0.
 * epi: 0 -> out fp16 = acc+bias; 1 -> out fp16 = QuickGELU(acc+bias); 5 -> out fp32 = acc+bias;
 *      6 -> out fp16 += acc+bias (sum in fp32, one rounding: the encoders' fp16 residual
 *      stream; no folded LayerNorm: rowstat / colsum NULL).  bias nullable (fp32).  fp16
 *      outputs: ldc % 8 == 0 (< 2^24), 16-byte aligned out. */
int reidmi_gemm_f16(int epi, const void* A, int64_t lda, const void* W, int64_t ldw, int64_t M, int64_t N, int64_t K,
                    const float* bias, const void* rowstat, const float* colsum, void* out, int64_t ldc, void* stream);

/* The product's timing hook (part of the product ABI on purpose; not an A/B variant — those live
 * in libreidmi_tools.so, reidmi_tools.h).  Measurement hooks: live timing of the GEMM launches (HIP events recorded on the launch stream
 * around each GEMM, including those inside reidmi_vit_forward / reidmi_text_forward), which is
 * how bench.py measures the dominant kernel's average launch time over its timed steps (the
 * roofline `achieved`; no other interface reaches a kernel inside the forward).  Off by
 * default: a disabled hook costs one branch per GEMM launch and records nothing.
 * collect: epi = GEMM epilogue id (-1 = all); returns summed device ms, launch count,
 * algorithmic FLOPs (2MNK) and clears the record. */
int reidmi_prof_enable(int on);
int reidmi_prof_collect(int epi, double* total_ms, int64_t* count, double* flops);
/* Same, counting only launches of >= min_flops (e.g. the full-batch launches of a kernel,
 * so that the average matches that kernel's row in a rocprofv3 --stats summary). */
int reidmi_prof_collect_min(int epi, double min_flops, double* total_ms, int64_t* count, double* flops);

/* Key padding used for an L-token sequence by the attention kernel (rows of v^T). */
int reidmi_attn_lpad(int L);

/* softmax(Q K^T / 8 [+causal]) V per (sequence, head): the SDPA of nn.MultiheadAttention
 * (custom_clip_model.py:22-24; causal text mask maple.py:956-962).  q,k [nseq*H][L][64],
 * vt [nseq*H][64][reidmi_attn_lpad(L)], o [nseq*L][H*64]; all fp16.  L <= 256. */
int reidmi_mhsa_f16(const void* q, const void* k, const void* vt, void* o, int64_t nseq, int L, int H, int causal,
                     void* stream);

/* LayerNorm over rows of width W in {512,768,1024} (fp32 math, eps) — custom_clip_model.py:43-49.
 * Row r of the output reads input row row_idx ? row_idx[r] : r.  y32 / y16 (fp16) nullable. */
int reidmi_layernorm(const float* x, int64_t rows, int64_t ldx, const int32_t* row_idx, int64_t W,
                     const float* gamma, const float* beta, float eps, float* y32, int64_t ldy32, void* y16,
                     int64_t ldy16, void* stream);

/* The encoder's LayerNorm-fold pieces, exported for tests.  row_stats_f16: st [rows] float2 =
 * (rstd, -mean*rstd) (eps 1e-5) of fp16 rows x [rows][ldx] (W = 512 | 768 | 1024), from a
 * pass over x (pst == NULL) or combined from 64-column partials pst [W/64][rows] float2.
 * gemm_f16_resid_partials: the residual GEMM (epi 6: out = half(out + A W^T + bias)) that
 * also writes those partials of the updated rows, pst[n/64 * M + m] (N % 64 == 0). */
int reidmi_row_stats_f16(const void* x, int64_t rows, int64_t ldx, int64_t W, const void* pst, void* st,
                         void* stream);
int reidmi_gemm_f16_resid_partials(const void* A, int64_t lda, const void* Wt, int64_t ldw, int64_t M, int64_t N,
                                   int64_t K, const float* bias, void* out, int64_t ldc, void* pst, void* stream);

/* Prompt construction — coop.PromptLearner.forward (coop.py:95-110) /
 * maple.VLPromptLearner.construct_prompts (maple.py:57-90): out [B][P+C+S][W] fp32 with
 * out[b] = cat(prefix [P][W], ctx[label[b]] [C][W] of ctx [ncls][C][W], suffix [S][W]).
 * W % 4 == 0.  bad_label (nullable device int32) is set to 1 for a label outside [0, ncls). */
int reidmi_prompt_build(const float* prefix, int P, const float* ctx, int C, const int64_t* label, int64_t ncls,
                        const float* suffix, int S, int64_t B, int W, float* out, int32_t* bad_label, void* stream);

/* Per-block weights of a CLIP transformer block (ResidualAttentionBlock,
 * custom_clip_model.py:8-29 / ResidualAttentionBlock_IVLP, maple.py:579-644).
 * Matrices in PyTorch [out][in] layout, vectors fp32.  ln_1 / ln_2 are folded into the
 * GEMM they feed:
 *   qkv_w = fp16(in_proj_weight * ln_1.weight[None, :]), qkv_b = in_proj_bias + in_proj_weight @ ln_1.bias,
 *   qkv_s[n] = sum_k qkv_w[n][k] (of the fp16 values, summed in double);
 *   fc1_w / fc1_b / fc1_s likewise from mlp.c_fc and ln_2.
 * out_w, fc2_w fp16.  ln1_w ... ln2_b are kept for reference (not read by the kernels).
 * prompt: IVLP VPT_shallow [n_ctx][W] (fp32) that replaces the prompt rows before this
 * block, or NULL. */
typedef struct reidmi_block_weights {
    const float* ln1_w;
    const float* ln1_b;
    const void* qkv_w;
    const float* qkv_b;
    const void* out_w;
    const float* out_b;
    const float* ln2_w;
    const float* ln2_b;
    const void* fc1_w;
    const float* fc1_b;
    const void* fc2_w;
    const float* fc2_b;
    const float* prompt;
    const float* qkv_s;
    const float* fc1_s;
} reidmi_block_weights;

/* Vision tower: custom_clip_model.VisionTransformer (custom_clip_model.py:57-100) and the
 * IVLP variant maple.VisionTransformer (maple.py:722-785) when n_ctx > 0.
 * conv_w: conv1.weight [W][3*P*P] flattened (c,ky,kx) and zero-padded to kpad (multiple of
 * 64), fp16.  proj_t: proj^T [out_dim][W] fp16.  blocks: HOST array of `layers` entries. */
typedef struct reidmi_vit_weights {
    int32_t width, layers, heads, patch, stride, out_dim, grid_h, grid_w, n_ctx, kpad;
    const void* conv_w;
    const float* class_emb;
    const float* pos_emb;
    const float* ln_pre_w;
    const float* ln_pre_b;
    const float* ln_post_w;
    const float* ln_post_b;
    const void* proj_t;
    const float* vpt;
    const reidmi_block_weights* blocks;
} reidmi_vit_weights;

/* Workspace bytes for reidmi_vit_forward at batch B (full = 0: CLS outputs only). */
int64_t reidmi_vit_workspace_bytes(const reidmi_vit_weights* w, int64_t B, int full);

/* encode_image: runs resblocks[:11] then resblocks[11] (custom_clip_model.py:91-92, also for
 * deeper towers), ln_post and proj.  images [B][3][H][Wimg] fp32 (images_f16 = 0) or fp16,
 * already normalised.  tta (nullable, device int32 [B][2]): apply the augmented loader's
 * flip + Pad((10,5)) + crop at (top, left) on the fly (data_prepare.py:263-270).
 * full = 0: out_x12 [B][W] = ln_post(x12)[:,0], out_proj [B][E] = (x12 @ proj)[:,0],
 *           out_x11 [B][W] = x11[:,0] (nullable)          (zero_shot_learning.py:84-87)
 * full = 1: out_x12 [B][L][W], out_proj [B][L][E], out_x11 [B][L][W] (nullable)
 *           — the (x11, x12, xproj) triple of encode_image. */
int reidmi_vit_forward(const reidmi_vit_weights* w, const void* images, int images_f16, int64_t B, int H,
                       int Wimg, const int32_t* tta, int full, float* out_x12, float* out_proj, float* out_x11,
                       void* ws, int64_t ws_bytes, void* stream);

/* Text tower: CLIP.encode_text (maple.py:971-984) from token ids, or
 * text_encoder.TextEncoder.forward (text_encoder.py:14-24) from pre-embedded prompts.
 * tok_emb [vocab][W] fp32, pos_emb [ctx][W] fp32, proj_t = text_projection^T [E][W] fp16. */
typedef struct reidmi_text_weights {
    int32_t width, layers, heads, ctx, vocab, out_dim, n_ctx;
    const float* tok_emb;
    const float* pos_emb;
    const float* ln_final_w;
    const float* ln_final_b;
    const void* proj_t;
    const reidmi_block_weights* blocks;
} reidmi_text_weights;

/* Workspace for N rows at the full ctx (an upper bound for any ctx_used). */
int64_t reidmi_text_workspace_bytes(const reidmi_text_weights* w, int64_t N);

/* tokens: device int64 [N][ctx] (always needed: the EOT row is tokens.argmax(-1)).
 * prompts: device fp32 [N][ctx][W] or NULL (then x = tok_emb[tokens]).  out [N][E] fp32.
 * ctx_used: 0 = all ctx positions; else run on the first ctx_used positions only, which
 * gives the same output when every row's EOT position (argmax) and IVLP prompt rows are
 * < ctx_used (causal mask: rows past the EOT never reach it); n_ctx < ctx_used <= ctx. */
int reidmi_text_forward(const reidmi_text_weights* w, const int64_t* tokens, const float* prompts, int64_t N,
                        int ctx_used, float* out, void* ws, int64_t ws_bytes, void* stream);

/* ------------------------------------------------ weight packing (checkpoint boundary, §8b)
 *
 * From the reference's fp32 tensors on the device, in its key layout, to a runnable tower whose
 * device data all lives in one caller-owned buffer (256-byte aligned, reidmi_*_pack_bytes):
 * CLIP-ReID checkpoints hold the vision tower under `image_encoder.*` (utils.py:169-221, loaded
 * into custom_clip_model.VisionTransformer) and the text tower under `text_encoder.*`
 * (zero_shot_learning.py:28-35, loaded into the CLIP text tower); strip the prefix and pass the
 * tensors below.  Packing (the definitions multimodal_reid_amd.model uses, pack.hip): ln_1 / ln_2
 * folded into in_proj / c_fc (W' = fp16(fp32(W gamma)), s = sum of W' rows, b' = fp32(b + W beta)
 * with a compensated fp64 sum), the other matrices cast to fp16 (utils.py:145-166 convert_weights),
 * conv1 flattened and zero-padded to a multiple of 64, proj / text_projection transposed; fp32
 * vectors copied.  Stream-ordered; the sources may be freed once the stream passes the call.
 * out_blocks: HOST array of `layers` entries that out->blocks will point to (keep it alive). */
typedef struct reidmi_block_src {  /* transformer.resblocks.{i}.* */
    const float* ln_1_w;           /* ln_1.weight [W] */
    const float* ln_1_b;           /* ln_1.bias [W] */
    const float* in_proj_w;        /* attn.in_proj_weight [3W][W] */
    const float* in_proj_b;        /* attn.in_proj_bias [3W] */
    const float* out_proj_w;       /* attn.out_proj.weight [W][W] */
    const float* out_proj_b;       /* attn.out_proj.bias [W] */
    const float* ln_2_w;           /* ln_2.weight [W] */
    const float* ln_2_b;           /* ln_2.bias [W] */
    const float* c_fc_w;           /* mlp.c_fc.weight [4W][W] */
    const float* c_fc_b;           /* mlp.c_fc.bias [4W] */
    const float* c_proj_w;         /* mlp.c_proj.weight [W][4W] */
    const float* c_proj_b;         /* mlp.c_proj.bias [W] */
    const float* vpt_shallow;      /* IVLP VPT_shallow [n_ctx][W] (maple.py:617-644), or NULL */
} reidmi_block_src;

/* Vision tower keys (custom_clip_model.py:57-76; maple.py:722-753 for IVLP).  The positional
 * embedding must already be at the (grid_h, grid_w) grid of the stride-12 patches (CLIP-ReID
 * checkpoints are; an OpenAI 224 x 224 grid goes through utils.resize_pos_embed first,
 * utils.py:111-125).  blocks: HOST array of `layers` entries. */
typedef struct reidmi_vit_src {
    int32_t width, layers, patch, stride, out_dim, grid_h, grid_w, n_ctx;
    const float* conv1_w;               /* conv1.weight [W][3][P][P] */
    const float* class_embedding;       /* [W] */
    const float* positional_embedding;  /* [1 + grid_h * grid_w][W] */
    const float* ln_pre_w;
    const float* ln_pre_b;
    const float* ln_post_w;
    const float* ln_post_b;
    const float* proj;                  /* [W][out_dim] */
    const float* vpt;                   /* VPT [n_ctx][W] or NULL */
    const reidmi_block_src* blocks;
} reidmi_vit_src;

/* Text tower keys of CLIP (maple.py:929-984): token_embedding.weight, positional_embedding,
 * transformer.resblocks.*, ln_final.*, text_projection.  blocks: HOST array of `layers`. */
typedef struct reidmi_text_src {
    int32_t width, layers, ctx, vocab, out_dim, n_ctx;
    const float* token_embedding;       /* [vocab][W] */
    const float* positional_embedding;  /* [ctx][W] */
    const float* ln_final_w;
    const float* ln_final_b;
    const float* text_projection;       /* [W][out_dim] */
    const reidmi_block_src* blocks;
} reidmi_text_src;

/* Buffer bytes for the packed tower (-1 on bad shapes). */
int64_t reidmi_vit_pack_bytes(const reidmi_vit_src* src);
int reidmi_vit_weights_pack(const reidmi_vit_src* src, void* buf, int64_t buf_bytes, reidmi_vit_weights* out,
                            reidmi_block_weights* out_blocks, void* stream);
int64_t reidmi_text_pack_bytes(const reidmi_text_src* src);
int reidmi_text_weights_pack(const reidmi_text_src* src, void* buf, int64_t buf_bytes, reidmi_text_weights* out,
                             reidmi_block_weights* out_blocks, void* stream);

/* -------------------------------------------------------- inference glue (G1) */

/* zeroshot_classifier (zero_shot_learning.py:42-48): out[c] = normalize(mean over rows
 * [offsets[c], offsets[c+1]) of normalize(feats[row])).  feats [rows][E], offsets device
 * int64 [ncls+1], out [ncls][E]; all fp32. */
int reidmi_class_mean_normalize(const float* feats, const int64_t* offsets, int64_t ncls, int64_t E, float* out,
                                void* stream);

/* zero_shot_learning.py:93,121-126 (non-mm): emb[b] = (cat(x12a,pa) + cat(x12b,pb)) / 2,
 * fp32 [B][W+E] with row stride lde. */
int reidmi_feature_tta_avg(const float* x12a, const float* pa, const float* x12b, const float* pb, int64_t B,
                           int64_t W, int64_t E, float* emb, int64_t lde, void* stream);

/* zero_shot_learning.py:116-122 (mm): emb[b] = cat((x12a+x12b)/2,
 * softmax((1/0.07) * normalize((pa+pb)/2) @ zs^T)), zs [ncls][E] fp32. */
int reidmi_feature_tta_mm(const float* x12a, const float* pa, const float* x12b, const float* pb, const float* zs,
                          int64_t B, int64_t W, int64_t E, int64_t ncls, float* emb, int64_t lde, void* stream);

/* ---------------------------------------------------- test-time transforms (§8f) */

/* transforms.Resize((oh, ow)) -> ToTensor() -> Normalize(mean, std)  — data_prepare.py:257-261
 * (the reference's test transform, applied per image in reidDataset.__getitem__,
 * data_prepare.py:87-92) on a packed batch of decoded RGB images; bit-exact with
 * PIL.Image.resize(BILINEAR) (Pillow 12.2, see oracle/transforms_oracle.c).  JPEG decode
 * stays on the host.
 * pix: device, concatenated HWC uint8 images; meta: device int64 [B][3] = (byte offset of
 * the image in pix, h, w) with 0 < h <= max_h, 0 < w <= max_w (images outside are skipped);
 * mean, stdv: HOST float[3]; out: device [B][3][oh][ow] (ow % 4 == 0), out_dtype 0 = fp32, 1 = fp16 (RNE).
 * The flip / pad / crop of the TTA loader (data_prepare.py:263-270) is applied on these
 * outputs by the encoder (reidmi_vit_forward's tta offsets). */
int reidmi_preprocess_u8(const uint8_t* pix, const int64_t* meta, int64_t B, int max_h, int max_w, int oh, int ow,
                         const float* mean, const float* stdv, int out_dtype, void* out, void* stream);

/* On-chip bytes one workgroup of reidmi_preprocess_u8 needs for sources up to max_h x max_w
 * (the call fails above 160 KiB: resize such images on the host first). */
int reidmi_preprocess_lds_size(int oh, int ow, int max_h, int max_w, int64_t* bytes);

/* ---------------------------------------------------------------- JPEG decode (§8f) */

/* Image.open(path).convert("RGB") — data_prepare.py:87-92 (reidDataset.__getitem__, run in the
 * DataLoader workers of data_prepare.py:275-283) — for a batch of JPEG files, bit-exact with
 * Pillow 12.2 / libjpeg-turbo defaults (islow IDCT, fancy upsampling).  Supported: baseline /
 * extended-sequential Huffman, 8-bit, one scan, grayscale or 3 components at 4:4:4, 4:2:2,
 * 4:2:0.  Two steps:
 *
 * reidmi_jpeg_plan (HOST only, no GPU): parses the headers of files[offsets[i] .. offsets[i+1])
 * (host bytes, offsets int64 [B+1]) and writes
 *   status int32 [B]  0 ok, 1 not a JPEG / truncated, 2 progressive / lossless / arithmetic /
 *                     12-bit / multi-scan, 3 component layout, 4 bad tables;
 *   meta int64 [B][3] (byte offset in the decoded batch, h, w) — the `meta` of
 *                     reidmi_preprocess_u8; zeros for images with status != 0;
 *   info int64 [10]   plan bytes, workspace bytes, decoded bytes, max h, max w, images with
 *                     status != 0, coefficient count, distinct Huffman tables, largest
 *                     per-image plane bytes, B;
 *   plan              when plan != NULL and plan_capacity >= info[0]: a position-independent
 *                     blob the caller copies to the device (call once with plan = NULL to size it).
 *
 * reidmi_jpeg_decode (stream-ordered): files = the same bytes on the DEVICE, plan = the plan on
 * the device, info = the HOST info[10] of the plan call (B must equal info[9]); ws >= info[1]
 * bytes; pix >= info[2] bytes receives the HWC uint8 images; err int32 [B] (device) = the plan
 * status, or 5 where the entropy-coded data does not decode (that image's coefficients are
 * then zero). */
int reidmi_jpeg_plan(const uint8_t* files, const int64_t* offsets, int64_t B, void* plan, int64_t plan_capacity,
                     int64_t* meta, int32_t* status, int64_t* info);
int reidmi_jpeg_decode(const uint8_t* files, const void* plan, const int64_t* info, int64_t B, void* ws,
                       int64_t ws_bytes, uint8_t* pix, int32_t* err, void* stream);

/* ---------------------------------------------------------------- loader file reads (§8f) */

/* The file side of reidDataset.__getitem__ (data_prepare.py:89 `Image.open(path)` in 4
 * DataLoader workers, data_prepare.py:275-283): one batch of encoded files gathered into ONE
 * caller-owned (pinned) host buffer by `nthreads` host threads (<= 0: up to 16), byte ranges
 * split evenly over the threads.  HOST only, no GPU.
 *
 * reidmi_files_size: sizes[i] = byte size of paths[i] (UTF-8 / file-system encoded, NUL-ended),
 *   or -1 where it cannot be opened.
 * reidmi_files_read: dst[offsets[i] .. offsets[i+1]) = the contents of paths[i]; status[i] = 0,
 *   1 (cannot open / read error) or 2 (the size differs from offsets[i+1] - offsets[i]).
 * reidmi_bytes_gather: dst[offsets[i] .. offsets[i+1]) = srcs[i][0 .. offsets[i+1] - offsets[i])
 *   (in-memory files, e.g. Python bytes objects).
 * Each returns an error only for bad arguments; per-file problems go to sizes / status. */
int reidmi_files_size(const char* const* paths, int64_t n, int64_t* sizes, int nthreads);
int reidmi_files_read(const char* const* paths, int64_t n, const int64_t* offsets, uint8_t* dst, int32_t* status,
                      int nthreads);
int reidmi_bytes_gather(const void* const* srcs, int64_t n, const int64_t* offsets, uint8_t* dst, int nthreads);

#ifdef __cplusplus
}
#endif
#endif /* REIDMI_H */
