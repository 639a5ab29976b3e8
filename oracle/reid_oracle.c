/*
 * reid_oracle.c — CPU restatement of the CLIP-ReID retrieval back end.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this (as the checker / the timed CPU baseline).  The
 * product path (libreidmi.so) never links, loads or falls back to it.
 *
 * It restates, function by function, the reference numpy/torch back end:
 *   evaluate.py:7-13   euclidean_distance          -> orc_distmat
 *   evaluate.py:114    F.normalize(p=2, dim=1)      -> orc_l2norm
 *   evaluate.py:29-88  eval_func (per-query part)   -> orc_eval_rows
 *   reranking.py:29-100 re_ranking (R2..R7)         -> orc_rerank_from_dist
 * Pinned against fixtures produced by the reference itself in this container
 * (tests/golden/make_goldens.py): eval_func and re_ranking(only_local=True) are
 * reproduced bit-exactly (ties canonicalised stable-by-index on both sides).
 *
 * Arithmetic definitions shared with the HIP kernels (bit-exact contract):
 *  - dot / squared norm: fmaf chain over k ascending (what v_mfma_f32_32x32x2_f32
 *    computes); distance = (qq + gg) - 2*dot.
 *  - numpy float32 exp (AVX512F/AVX2 simd_exp_f32, numpy 2.2.6): Cody-Waite + 5/2
 *    rational polynomial, constants pinned by probing numpy here (2e6/2e6 match).
 *  - numpy float32 pairwise sum (PW_BLOCKSIZE 128, 8 accumulators).
 *  - numpy float16 ufuncs: op in float32 then round-to-nearest-even to half.
 * Build with -ffp-contract=off (no implicit FMA) — see oracle/Makefile.
 *
 * Threads (orc_set_threads, pthreads): rows / queries / column blocks are independent, so
 * every parallel loop computes exactly what the serial one does (bench.py times the CPU
 * baseline with the host's cores).  The distance kernel vectorises across gallery columns
 * with AVX2 FMA (IEEE fused multiply-add == fmaf, same k order) when the CPU has it.
 */
#include <immintrin.h>
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------- threads ---- */
static int g_threads = 1;
void orc_set_threads(int n) { g_threads = n < 1 ? 1 : (n > 256 ? 256 : n); }
int orc_get_threads(void) { return g_threads; }

typedef void (*range_fn)(int64_t lo, int64_t hi, int tid, void* ctx);
typedef struct {
    range_fn fn;
    void* ctx;
    int64_t n, chunk;
    int64_t* next;
    int tid;
} job_t;

static void* run_job(void* p) {
    job_t* j = (job_t*)p;
    for (;;) {
        int64_t lo = __atomic_fetch_add(j->next, j->chunk, __ATOMIC_RELAXED);
        if (lo >= j->n) break;
        int64_t hi = lo + j->chunk < j->n ? lo + j->chunk : j->n;
        j->fn(lo, hi, j->tid, j->ctx);
    }
    return NULL;
}

/* fn(lo, hi, tid, ctx) over [0, n) in dynamic chunks; tid < orc_get_threads() */
static void par_for(int64_t n, int64_t chunk, range_fn fn, void* ctx) {
    int t = g_threads;
    if (chunk < 1) chunk = 1;
    if ((int64_t)t > (n + chunk - 1) / chunk) t = (int)((n + chunk - 1) / chunk);
    if (t <= 1) {
        if (n > 0) fn(0, n, 0, ctx);
        return;
    }
    int64_t next = 0;
    pthread_t th[256];
    job_t jobs[256];
    for (int i = 0; i < t; i++) {
        jobs[i] = (job_t){fn, ctx, n, chunk, &next, i};
        if (i > 0) pthread_create(&th[i], NULL, run_job, &jobs[i]);
    }
    run_job(&jobs[0]);
    for (int i = 1; i < t; i++) pthread_join(th[i], NULL);
}

/* ---------------------------------------------------------------- fp16 ---- */
uint16_t orc_f2h(float f) {
    uint32_t x; memcpy(&x, &f, 4);
    uint32_t sign = (x >> 16) & 0x8000u;
    uint32_t ax = x & 0x7fffffffu;
    if (ax >= 0x7f800000u) return (uint16_t)(sign | 0x7c00u | (ax > 0x7f800000u ? 0x200u : 0));
    if (ax >= 0x477ff000u) return (uint16_t)(sign | 0x7c00u); /* rounds to >= 65520 -> inf */
    if (ax < 0x38800000u) { /* subnormal half (or zero) */
        if (ax < 0x33000000u) return (uint16_t)sign; /* < 2^-25 -> 0 (tie at 2^-25 -> even 0) */
        uint32_t e = ax >> 23, m = (ax & 0x7fffffu) | 0x800000u;
        /* value = m * 2^(e-150); in units of the half subnormal step 2^-24: m >> (126 - e) */
        uint32_t shift = 126 - e;
        uint32_t q = m >> shift, r = m & ((1u << shift) - 1), half = 1u << (shift - 1);
        if (r > half || (r == half && (q & 1))) q++;
        return (uint16_t)(sign | q);
    }
    uint32_t e = (ax >> 23) - 112; /* rebias 127 -> 15 */
    uint32_t m = ax & 0x7fffffu;
    uint32_t q = (e << 10) | (m >> 13), r = m & 0x1fffu;
    if (r > 0x1000u || (r == 0x1000u && (q & 1))) q++;
    return (uint16_t)(sign | q);
}

float orc_h2f(uint16_t h) {
    uint32_t sign = (uint32_t)(h & 0x8000u) << 16, e = (h >> 10) & 0x1fu, m = h & 0x3ffu, x;
    if (e == 0) {
        if (m == 0) x = sign;
        else { float f = (float)m * 5.9604644775390625e-08f; memcpy(&x, &f, 4); x |= sign; }
    } else if (e == 31) x = sign | 0x7f800000u | (m << 13);
    else x = sign | ((e + 112) << 23) | (m << 13);
    float f; memcpy(&f, &x, 4); return f;
}

/* ------------------------------------------------------- numpy float32 exp */
float orc_np_expf(float x) {
    if (x != x) return x;
    if (x > 88.72283935546875f) return INFINITY;
    if (x < -103.97208404541015625f) return 0.0f;
    const float log2e = 1.442695040888963407359924681001892137f;
    float quad = rintf(x * log2e);
    float r = fmaf(quad, -6.93145752e-1f, x);
    r = fmaf(quad, -1.42860677e-6f, r);
    float num = fmaf(5.082762527590693718096e-04f, r, 6.757896990527504603057e-03f);
    num = fmaf(num, r, 5.114512081637298353406e-02f);
    num = fmaf(num, r, 2.473615434895520810817e-01f);
    num = fmaf(num, r, 7.257664613233124478488e-01f);
    num = fmaf(num, r, 9.999999999980870924916e-01f);
    float den = fmaf(2.159509375685829852307e-02f, r, -2.742335390411667452936e-01f);
    den = fmaf(den, r, 1.0f);
    return ldexpf(num / den, (int)quad);
}

/* ---------------------------------------------------- numpy pairwise sums */
float orc_pairwise_f32(const float* a, int64_t n) {
    if (n < 8) {
        float res = 0.0f;
        for (int64_t i = 0; i < n; i++) res += a[i];
        return res;
    } else if (n <= 128) {
        float r[8];
        for (int j = 0; j < 8; j++) r[j] = a[j];
        int64_t i;
        for (i = 8; i < n - (n % 8); i += 8)
            for (int j = 0; j < 8; j++) r[j] += a[i + j];
        float res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; i++) res += a[i];
        return res;
    }
    int64_t n2 = n / 2; n2 -= n2 % 8;
    return orc_pairwise_f32(a, n2) + orc_pairwise_f32(a + n2, n - n2);
}

double orc_pairwise_f64(const double* a, int64_t n) {
    if (n < 8) {
        double res = 0.0;
        for (int64_t i = 0; i < n; i++) res += a[i];
        return res;
    } else if (n <= 128) {
        double r[8];
        for (int j = 0; j < 8; j++) r[j] = a[j];
        int64_t i;
        for (i = 8; i < n - (n % 8); i += 8)
            for (int j = 0; j < 8; j++) r[j] += a[i + j];
        double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; i++) res += a[i];
        return res;
    }
    int64_t n2 = n / 2; n2 -= n2 % 8;
    return orc_pairwise_f64(a, n2) + orc_pairwise_f64(a + n2, n - n2);
}

/* --------------------------------------------------------- l2 / distmat */
static float sqnorm(const float* x, int64_t d) {
    float acc = 0.0f;
    for (int64_t k = 0; k < d; k++) acc = fmaf(x[k], x[k], acc);
    return acc;
}

/* F.normalize(x, p=2, dim=1): x / max(||x||, 1e-12)   (evaluate.py:114) */
void orc_l2norm(const float* x, float* y, int64_t n, int64_t d) {
    for (int64_t i = 0; i < n; i++) {
        float nrm = sqrtf(sqnorm(x + i * d, d));
        if (nrm < 1e-12f) nrm = 1e-12f;
        for (int64_t k = 0; k < d; k++) y[i * d + k] = x[i * d + k] / nrm;
    }
}

/* ||q||^2 + ||g||^2 - 2 q.g   (evaluate.py:7-13; reranking.py:36-41): per pair an fmaf chain
 * over k ascending, then fmaf(-2, dot, qq + gg). */
typedef struct {
    const float *q, *g;
    int64_t Q, G, D;
    const float *qq, *gg;
    float* out;
} dist_ctx;

static void sqnorm_rows(int64_t lo, int64_t hi, int tid, void* c) {
    (void)tid;
    float** a = (float**)c;
    const float* x = a[0];
    float* o = a[1];
    int64_t d = (int64_t)(intptr_t)a[2];
    for (int64_t i = lo; i < hi; i++) o[i] = sqnorm(x + i * d, d);
}

static void dist_scalar(int64_t lo, int64_t hi, int tid, void* c) {
    (void)tid;
    const dist_ctx* x = (const dist_ctx*)c;
    for (int64_t i = lo; i < hi; i++)
        for (int64_t j = 0; j < x->G; j++) {
            float acc = 0.0f;
            const float* a = x->q + i * x->D; const float* b = x->g + j * x->D;
            for (int64_t k = 0; k < x->D; k++) acc = fmaf(a[k], b[k], acc);
            x->out[i * x->G + j] = fmaf(-2.0f, acc, x->qq[i] + x->gg[j]);
        }
}

/* one block of DB gallery columns: transposed into gT [D][DB], then 4 query rows x 16
 * columns per register tile (8 accumulators, k ascending: the fmaf chain of every pair) */
#define DB 256
__attribute__((target("avx2,fma"))) static void dist_avx2(int64_t lo, int64_t hi, int tid, void* c) {
    (void)tid;
    const dist_ctx* x = (const dist_ctx*)c;
    const int64_t D = x->D, G = x->G, Q = x->Q;
    float* gT = (float*)aligned_alloc(64, sizeof(float) * (size_t)(D * DB));
    for (int64_t jb = lo; jb < hi; jb++) {
        const int64_t j0 = jb * DB, nj = G - j0 < DB ? G - j0 : DB;
        for (int64_t t = 0; t < DB; t++)
            for (int64_t k = 0; k < D; k++) gT[k * DB + t] = t < nj ? x->g[(j0 + t) * D + k] : 0.0f;
        for (int64_t i0 = 0; i0 < Q; i0 += 4) {
            const int64_t ni = Q - i0 < 4 ? Q - i0 : 4;
            const float* a[4];
            for (int r = 0; r < 4; r++) a[r] = x->q + (i0 + (r < ni ? r : 0)) * D;
            for (int64_t t0 = 0; t0 < nj; t0 += 16) {
                __m256 acc[4][2];
                for (int r = 0; r < 4; r++) acc[r][0] = acc[r][1] = _mm256_setzero_ps();
                for (int64_t k = 0; k < D; k++) {
                    const __m256 b0 = _mm256_load_ps(gT + k * DB + t0), b1 = _mm256_load_ps(gT + k * DB + t0 + 8);
                    for (int r = 0; r < 4; r++) {
                        const __m256 av = _mm256_set1_ps(a[r][k]);
                        acc[r][0] = _mm256_fmadd_ps(av, b0, acc[r][0]);
                        acc[r][1] = _mm256_fmadd_ps(av, b1, acc[r][1]);
                    }
                }
                float tmp[16];
                for (int r = 0; r < ni; r++) {
                    _mm256_storeu_ps(tmp, acc[r][0]);
                    _mm256_storeu_ps(tmp + 8, acc[r][1]);
                    for (int64_t t = 0; t < 16 && t0 + t < nj; t++)
                        x->out[(i0 + r) * G + j0 + t0 + t] = fmaf(-2.0f, tmp[t], x->qq[i0 + r] + x->gg[j0 + t0 + t]);
                }
            }
        }
    }
    free(gT);
}

void orc_distmat(const float* q, const float* g, int64_t Q, int64_t G, int64_t D, float* out) {
    float* qq = (float*)malloc(sizeof(float) * (size_t)(Q > 0 ? Q : 1));
    float* gg = (float*)malloc(sizeof(float) * (size_t)(G > 0 ? G : 1));
    void* a1[3] = {(void*)q, qq, (void*)(intptr_t)D};
    void* a2[3] = {(void*)g, gg, (void*)(intptr_t)D};
    par_for(Q, 256, sqnorm_rows, a1);
    par_for(G, 256, sqnorm_rows, a2);
    dist_ctx c = {q, g, Q, G, D, qq, gg, out};
    __builtin_cpu_init();
    if (__builtin_cpu_supports("avx2") && __builtin_cpu_supports("fma"))
        par_for((G + DB - 1) / DB, 1, dist_avx2, &c);
    else
        par_for(Q, 4, dist_scalar, &c);
    free(qq);
    free(gg);
}

/* ---------------------------------------------------- stable argsort (rows) */
typedef struct { float v; int32_t i; } kv_t;
static int kv_cmp(const void* a, const void* b) {
    const kv_t* x = (const kv_t*)a; const kv_t* y = (const kv_t*)b;
    if (x->v < y->v) return -1;
    if (y->v < x->v) return 1;
    return (x->i > y->i) - (x->i < y->i);
}
/* argsort of one row; ties broken by index (== np.argsort(kind="stable")) */
static void argsort_row(const float* row, int64_t n, kv_t* tmp, int32_t* idx) {
    for (int64_t j = 0; j < n; j++) { tmp[j].v = row[j]; tmp[j].i = (int32_t)j; }
    qsort(tmp, (size_t)n, sizeof(kv_t), kv_cmp);
    for (int64_t j = 0; j < n; j++) idx[j] = tmp[j].i;
}

/* first k of the stable argsort of each row: a sorted insertion buffer of the k smallest
 * (value, index) keys (== the full stable sort's prefix) */
typedef struct {
    const float* x;
    int64_t G, k;
    int32_t* out;
} topk_ctx;

static int kv_less(float av, int32_t ai, float bv, int32_t bi) { return av < bv || (av == bv && ai < bi); }

static void topk_part(int64_t lo, int64_t hi, int tid, void* c) {
    (void)tid;
    const topk_ctx* t = (const topk_ctx*)c;
    kv_t* buf = (kv_t*)malloc(sizeof(kv_t) * (size_t)t->k);
    for (int64_t i = lo; i < hi; i++) {
        const float* row = t->x + i * t->G;
        int64_t n = 0;
        for (int64_t j = 0; j < t->G; j++) {
            const float v = row[j];
            if (n == t->k && !kv_less(v, (int32_t)j, buf[n - 1].v, buf[n - 1].i)) continue;
            int64_t p = n < t->k ? n++ : n - 1;
            while (p > 0 && kv_less(v, (int32_t)j, buf[p - 1].v, buf[p - 1].i)) { buf[p] = buf[p - 1]; p--; }
            buf[p].v = v;
            buf[p].i = (int32_t)j;
        }
        for (int64_t r = 0; r < t->k; r++) t->out[i * t->k + r] = buf[r].i;
    }
    free(buf);
}

void orc_topk_rows(const float* dist, int64_t Q, int64_t G, int64_t k, int32_t* out) {
    topk_ctx c = {dist, G, k, out};
    par_for(Q, 16, topk_part, &c);
}

/* ------------------------------------------------------------- eval_func */
/* Per-query part of eval_func (evaluate.py:40-80).  For each query:
 *   valid[q]  = any positive kept  (evaluate.py:61-63)
 *   first[q]  = 0-based position of the first match among kept items
 *   ap[q]     = AP exactly as numpy computes it (cumsum/arange*orig_cmc, pairwise sum / num_rel)
 *   nkept[q]  = number of kept gallery items (length of orig_cmc)            */
typedef struct {
    const float* dist;
    int64_t G;
    const int64_t *qp, *gp, *qc, *gc;
    int32_t* valid;
    int64_t *first, *nkept;
    double* ap;
} eval_ctx;

static void eval_part(int64_t lo, int64_t hi, int tid, void* c) {
    (void)tid;
    const eval_ctx* e = (const eval_ctx*)c;
    const int64_t G = e->G;
    kv_t* tmp = (kv_t*)malloc(sizeof(kv_t) * (size_t)G);
    int32_t* idx = (int32_t*)malloc(sizeof(int32_t) * (size_t)G);
    double* t = (double*)malloc(sizeof(double) * (size_t)G);
    for (int64_t q = lo; q < hi; q++) {
        argsort_row(e->dist + q * G, G, tmp, idx);
        int64_t n = 0, hits = 0, f = -1;
        for (int64_t j = 0; j < G; j++) {
            int32_t g = idx[j];
            if (e->gp[g] == e->qp[q] && e->gc[g] == e->qc[q]) continue; /* remove */
            int m = e->gp[g] == e->qp[q];
            if (m) { hits++; if (f < 0) f = n; }
            /* tmp_cmc = cumsum / arange(1..) ; * orig_cmc  (evaluate.py:74-78) */
            t[n] = m ? (double)hits / (double)(n + 1) : 0.0;
            n++;
        }
        e->nkept[q] = n;
        e->valid[q] = hits > 0;
        e->first[q] = f;
        e->ap[q] = hits > 0 ? orc_pairwise_f64(t, n) / (double)hits : 0.0;
    }
    free(tmp); free(idx); free(t);
}

void orc_eval_rows(const float* dist, int64_t Q, int64_t G, const int64_t* qp, const int64_t* gp,
                   const int64_t* qc, const int64_t* gc, int32_t* valid, int64_t* first, double* ap,
                   int64_t* nkept) {
    eval_ctx c = {dist, G, qp, gp, qc, gc, valid, first, nkept, ap};
    par_for(Q, 4, eval_part, &c);
}

/* ------------------------------------------------------------- re_ranking */
static int cmp_i32(const void* a, const void* b) {
    int32_t x = *(const int32_t*)a, y = *(const int32_t*)b;
    return (x > y) - (x < y);
}

/* k-reciprocal set of row i at depth kk (reranking.py:53-56 / 60-63):
 * forward = R[i, :kk+1]; keep forward[f] whose row R[forward[f], :kk+1] contains i. */
static int kreciprocal(const int32_t* R, int64_t ldr, int32_t i, int kk1, int32_t* out) {
    int n = 0;
    for (int f = 0; f < kk1; f++) {
        int32_t c = R[(int64_t)i * ldr + f];
        for (int b = 0; b < kk1; b++)
            if (R[(int64_t)c * ldr + b] == i) { out[n++] = c; break; }
    }
    return n;
}

/* re_ranking(..., local_distmat=D, only_local=True) — reranking.py:29-100 with
 * D the N x N original distance (rows/cols: queries then gallery).
 * one_minus_lambda_h = np.float16(1 - lambda) bits and lambda_f = np.float32(lambda): the
 * numpy weak-scalar conversions of reranking.py:95 (the caller makes them with numpy).
 * final: Q x (N-Q) float32.  Optional debug outputs (may be NULL):
 * rank_out N x K int32 (K = min(max(k1+1,k2), N)), vqe_out N x N fp16 bits, jac_out Q x N fp16 bits. */
typedef struct {
    const float* D;
    float* od;
    float* colmax;
    float* part;  /* [nchunk][N] partial column maxima */
    int64_t N, Q, K, nchunk;
    const int32_t* R;
    int kf, kh1, k2;
    uint16_t *V, *Vq;
    int64_t *ccnt, *cnt;  /* [nchunk][N+1] per-chunk column counts / positions; cnt [N+1] */
    int32_t* inv;
    uint16_t lam16;
    float lam_f;
    float* final_out;
    uint16_t* jac_out;
    uint16_t* tmin;  /* [threads][N] */
} rr_ctx;

static void rr_colmax(int64_t lo, int64_t hi, int tid, void* c) {
    (void)tid;
    rr_ctx* x = (rr_ctx*)c;
    const int64_t N = x->N;
    for (int64_t ch = lo; ch < hi; ch++) {
        float* m = x->part + ch * N;
        const int64_t r0 = N * ch / x->nchunk, r1 = N * (ch + 1) / x->nchunk;
        for (int64_t cc = 0; cc < N; cc++) m[cc] = x->D[r0 * N + cc];
        for (int64_t r = r0 + 1; r < r1; r++)
            for (int64_t cc = 0; cc < N; cc++) if (x->D[r * N + cc] > m[cc]) m[cc] = x->D[r * N + cc];
    }
}

static void rr_od(int64_t lo, int64_t hi, int tid, void* c) {
    (void)tid;
    rr_ctx* x = (rr_ctx*)c;
    const int64_t N = x->N;
    for (int64_t i = lo; i < hi; i++)
        for (int64_t j = 0; j < N; j++) x->od[i * N + j] = x->D[j * N + i] / x->colmax[i];
}

static void rr_v(int64_t lo, int64_t hi, int tid, void* c) {
    (void)tid;
    rr_ctx* x = (rr_ctx*)c;
    const int64_t N = x->N, K = x->K;
    const int kf = x->kf, kh1 = x->kh1;
    int32_t* kr = (int32_t*)malloc(sizeof(int32_t) * (size_t)kf);
    int32_t* ckr = (int32_t*)malloc(sizeof(int32_t) * (size_t)kh1);
    int32_t* exp_idx = (int32_t*)malloc(sizeof(int32_t) * (size_t)(kf + (int64_t)kf * kh1));
    float* w = (float*)malloc(sizeof(float) * (size_t)(kf + (int64_t)kf * kh1));
    for (int64_t i = lo; i < hi; i++) {
        int nk = kreciprocal(x->R, K, (int32_t)i, kf, kr);
        int ne = 0;
        for (int a = 0; a < nk; a++) exp_idx[ne++] = kr[a];
        for (int a = 0; a < nk; a++) {
            int nc = kreciprocal(x->R, K, kr[a], kh1, ckr);
            int inter = 0;
            for (int b = 0; b < nc; b++)
                for (int cc = 0; cc < nk; cc++) if (ckr[b] == kr[cc]) { inter++; break; }
            if ((double)inter > 2.0 / 3.0 * (double)nc)
                for (int b = 0; b < nc; b++) exp_idx[ne++] = ckr[b];
        }
        qsort(exp_idx, (size_t)ne, sizeof(int32_t), cmp_i32);
        int nu = 0;
        for (int a = 0; a < ne; a++) if (nu == 0 || exp_idx[a] != exp_idx[nu - 1]) exp_idx[nu++] = exp_idx[a];
        for (int a = 0; a < nu; a++) w[a] = orc_np_expf(-x->od[i * N + exp_idx[a]]);
        float s = orc_pairwise_f32(w, nu);
        for (int a = 0; a < nu; a++) x->V[i * N + exp_idx[a]] = orc_f2h(w[a] / s);
    }
    free(kr); free(ckr); free(exp_idx); free(w);
}

static void rr_qe(int64_t lo, int64_t hi, int tid, void* c) {
    (void)tid;
    rr_ctx* x = (rr_ctx*)c;
    const int64_t N = x->N;
    float* acc = (float*)malloc(sizeof(float) * (size_t)N);
    for (int64_t i = lo; i < hi; i++) {
        for (int64_t cc = 0; cc < N; cc++) acc[cc] = 0.0f;
        for (int r = 0; r < x->k2; r++) {
            const uint16_t* row = x->V + (int64_t)x->R[i * x->K + r] * N;
            for (int64_t cc = 0; cc < N; cc++) acc[cc] += orc_h2f(row[cc]);
        }
        for (int64_t cc = 0; cc < N; cc++) x->Vq[i * N + cc] = orc_f2h(acc[cc] / (float)x->k2);
    }
    free(acc);
}

static void rr_count(int64_t lo, int64_t hi, int tid, void* c) {
    (void)tid;
    rr_ctx* x = (rr_ctx*)c;
    const int64_t N = x->N;
    for (int64_t ch = lo; ch < hi; ch++) {
        int64_t* cn = x->ccnt + ch * (N + 1);
        for (int64_t cc = 0; cc <= N; cc++) cn[cc] = 0;
        for (int64_t r = N * ch / x->nchunk; r < N * (ch + 1) / x->nchunk; r++)
            for (int64_t cc = 0; cc < N; cc++) if (x->V[r * N + cc] & 0x7fffu) cn[cc]++;
    }
}

static void rr_fill(int64_t lo, int64_t hi, int tid, void* c) {
    (void)tid;
    rr_ctx* x = (rr_ctx*)c;
    const int64_t N = x->N;
    for (int64_t ch = lo; ch < hi; ch++) {
        int64_t* pos = x->ccnt + ch * (N + 1);  /* positions of this chunk's first entry per column */
        for (int64_t r = N * ch / x->nchunk; r < N * (ch + 1) / x->nchunk; r++)
            for (int64_t cc = 0; cc < N; cc++) if (x->V[r * N + cc] & 0x7fffu) x->inv[pos[cc]++] = (int32_t)r;
    }
}

static void rr_jaccard(int64_t lo, int64_t hi, int tid, void* c) {
    rr_ctx* x = (rr_ctx*)c;
    const int64_t N = x->N, Q = x->Q, G = N - Q;
    const uint16_t* V = x->V;
    uint16_t* tmin = x->tmin + (int64_t)tid * N;
    for (int64_t i = lo; i < hi; i++) {
        for (int64_t r = 0; r < N; r++) tmin[r] = 0;
        for (int64_t cc = 0; cc < N; cc++) {
            uint16_t vi = V[i * N + cc];
            if (!(vi & 0x7fffu)) continue;
            float fvi = orc_h2f(vi);
            for (int64_t p = x->cnt[cc]; p < x->cnt[cc + 1]; p++) {
                int32_t r = x->inv[p];
                float fvr = orc_h2f(V[(int64_t)r * N + cc]);
                float mn = fvr < fvi ? fvr : fvi;               /* np.minimum (fp16) */
                tmin[r] = orc_f2h(orc_h2f(tmin[r]) + mn);        /* fp16 + fp16 -> fp16 */
            }
        }
        for (int64_t r = 0; r < N; r++) {
            float t = orc_h2f(tmin[r]);
            uint16_t den = orc_f2h(2.0f - t);                       /* 2 - temp_min   */
            uint16_t qt = orc_f2h(t / orc_h2f(den));                /* temp_min / (.) */
            uint16_t jac = orc_f2h(1.0f - orc_h2f(qt));             /* 1 - (.)        */
            if (x->jac_out) x->jac_out[i * N + r] = jac;
            if (r >= Q) {
                /* R7: jaccard*(1-lambda) [fp16] + original_dist*lambda [fp32] (reranking.py:95) */
                float a = orc_h2f(orc_f2h(orc_h2f(jac) * orc_h2f(x->lam16)));
                float b = x->od[i * N + r] * x->lam_f;
                x->final_out[i * G + (r - Q)] = a + b;
            }
        }
    }
}

int orc_rerank_from_dist(const float* D, int64_t N, int64_t Q, int k1, int k2, uint16_t one_minus_lambda_h,
                         float lambda_f, float* final_out, int32_t* rank_out, uint16_t* vqe_out, uint16_t* jac_out) {
    rr_ctx x;
    memset(&x, 0, sizeof(x));
    x.D = D; x.N = N; x.Q = Q; x.k2 = k2; x.lam16 = one_minus_lambda_h; x.lam_f = lambda_f;
    x.final_out = final_out; x.jac_out = jac_out;
    x.nchunk = g_threads < N ? g_threads : N;
    /* R2: od = transpose(D / max(D, axis=0))  (reranking.py:46) */
    x.part = (float*)malloc(sizeof(float) * (size_t)(x.nchunk * N));
    par_for(x.nchunk, 1, rr_colmax, &x);
    x.colmax = (float*)malloc(sizeof(float) * (size_t)N);
    for (int64_t cc = 0; cc < N; cc++) {
        float m = x.part[cc];
        for (int64_t ch = 1; ch < x.nchunk; ch++) if (x.part[ch * N + cc] > m) m = x.part[ch * N + cc];
        x.colmax[cc] = m;
    }
    free(x.part);
    x.od = (float*)malloc(sizeof(float) * (size_t)(N * N));
    par_for(N, 64, rr_od, &x);
    /* initial_rank = argsort(od) (stable), first K columns (reranking.py:48) */
    int64_t K = k1 + 1 > k2 ? k1 + 1 : k2; if (K > N) K = N;
    x.K = K;
    int32_t* R = (int32_t*)malloc(sizeof(int32_t) * (size_t)(N * K));
    orc_topk_rows(x.od, N, N, K, R);
    x.R = R;
    if (rank_out) memcpy(rank_out, R, sizeof(int32_t) * (size_t)(N * K));
    x.kf = (int)(k1 + 1 < N ? k1 + 1 : N);
    int kh = (int)nearbyint((double)k1 / 2.0); /* int(np.around(k1/2)) (round half even) */
    x.kh1 = kh + 1 < N ? kh + 1 : (int)N;
    /* R3: V (dense fp16 bits), reranking.py:51-71 */
    x.V = (uint16_t*)calloc((size_t)(N * N), sizeof(uint16_t));
    par_for(N, 16, rr_v, &x);
    /* R4: query expansion (reranking.py:73-78) */
    if (k2 != 1) {
        x.Vq = (uint16_t*)malloc(sizeof(uint16_t) * (size_t)(N * N));
        par_for(N, 16, rr_qe, &x);
        free(x.V);
        x.V = x.Vq;
    }
    if (vqe_out) memcpy(vqe_out, x.V, sizeof(uint16_t) * (size_t)(N * N));
    /* R5: invIndex (reranking.py:80-82) as column lists, rows ascending (row chunks in order) */
    x.ccnt = (int64_t*)malloc(sizeof(int64_t) * (size_t)(x.nchunk * (N + 1)));
    par_for(x.nchunk, 1, rr_count, &x);
    x.cnt = (int64_t*)calloc((size_t)N + 1, sizeof(int64_t));
    for (int64_t cc = 0; cc < N; cc++) {
        int64_t tot = 0;
        for (int64_t ch = 0; ch < x.nchunk; ch++) tot += x.ccnt[ch * (N + 1) + cc];
        x.cnt[cc + 1] = x.cnt[cc] + tot;
    }
    for (int64_t cc = 0; cc < N; cc++) {
        int64_t p = x.cnt[cc];
        for (int64_t ch = 0; ch < x.nchunk; ch++) {
            const int64_t n = x.ccnt[ch * (N + 1) + cc];
            x.ccnt[ch * (N + 1) + cc] = p;
            p += n;
        }
    }
    x.inv = (int32_t*)malloc(sizeof(int32_t) * (size_t)(x.cnt[N] > 0 ? x.cnt[N] : 1));
    par_for(x.nchunk, 1, rr_fill, &x);
    /* R6 + R7: Jaccard (reranking.py:84-100) with fp16 sequential accumulation */
    x.tmin = (uint16_t*)malloc(sizeof(uint16_t) * (size_t)(g_threads * N));
    par_for(Q, 4, rr_jaccard, &x);
    free(x.colmax); free(x.od); free(R); free(x.V); free(x.ccnt); free(x.cnt); free(x.inv); free(x.tmin);
    return 0;
}

/* ------------------------------------------------- staged re_ranking (rows) */
/* The same R2-R7 as orc_rerank_from_dist, split into row-range stages over a symmetric
 * distance given as row blocks (the sharded product path's stage boundaries).
 * Test infrastructure: tests/test_rerank_sharded_gloo.py drives these under the product's
 * orchestration (multimodal_reid_amd/reranking.py staged_rerank). */

/* R2 for rows lo..hi: Drows [rows][N]; rowmax = row maxima (= column maxima, D symmetric,
 * reranking.py:46); R [rows][K] = stable argsort prefix of Drows[r] / rowmax[r]. */
void orc_rr_rank_rows(const float* Drows, int64_t rows, int64_t N, int64_t K, int32_t* R, float* rowmax) {
    float* od = (float*)malloc(sizeof(float) * (size_t)N);
    kv_t* tmp = (kv_t*)malloc(sizeof(kv_t) * (size_t)N);
    int32_t* idx = (int32_t*)malloc(sizeof(int32_t) * (size_t)N);
    for (int64_t r = 0; r < rows; r++) {
        const float* d = Drows + r * N;
        float m = d[0];
        for (int64_t j = 1; j < N; j++) if (d[j] > m) m = d[j];
        rowmax[r] = m;
        for (int64_t j = 0; j < N; j++) od[j] = d[j] / m;
        argsort_row(od, N, tmp, idx);
        memcpy(R + r * K, idx, sizeof(int32_t) * (size_t)K);
    }
    free(od); free(tmp); free(idx);
}

/* R3 for rows lo..hi (reranking.py:51-71): Drows [hi-lo][N] distances of those rows,
 * rowmax [N], R [N][K] (all rows).  Vrows [hi-lo][N] fp16 bits (dense). */
void orc_rr_v_rows(const float* Drows, const float* rowmax, const int32_t* R, int64_t N, int64_t K, int64_t lo,
                   int64_t hi, int k1, uint16_t* Vrows) {
    int kf = (int)(k1 + 1 < N ? k1 + 1 : N);
    int kh = (int)nearbyint((double)k1 / 2.0);
    int kh1 = kh + 1 < N ? kh + 1 : (int)N;
    int32_t* kr = (int32_t*)malloc(sizeof(int32_t) * (size_t)kf);
    int32_t* ckr = (int32_t*)malloc(sizeof(int32_t) * (size_t)kh1);
    int32_t* exp_idx = (int32_t*)malloc(sizeof(int32_t) * (size_t)(kf + (int64_t)kf * kh1));
    float* w = (float*)malloc(sizeof(float) * (size_t)(kf + (int64_t)kf * kh1));
    memset(Vrows, 0, sizeof(uint16_t) * (size_t)((hi - lo) * N));
    for (int64_t i = lo; i < hi; i++) {
        int nk = kreciprocal(R, K, (int32_t)i, kf, kr);
        int ne = 0;
        for (int a = 0; a < nk; a++) exp_idx[ne++] = kr[a];
        for (int a = 0; a < nk; a++) {
            int nc = kreciprocal(R, K, kr[a], kh1, ckr);
            int inter = 0;
            for (int b = 0; b < nc; b++)
                for (int c = 0; c < nk; c++) if (ckr[b] == kr[c]) { inter++; break; }
            if ((double)inter > 2.0 / 3.0 * (double)nc)
                for (int b = 0; b < nc; b++) exp_idx[ne++] = ckr[b];
        }
        qsort(exp_idx, (size_t)ne, sizeof(int32_t), cmp_i32);
        int nu = 0;
        for (int a = 0; a < ne; a++) if (nu == 0 || exp_idx[a] != exp_idx[nu - 1]) exp_idx[nu++] = exp_idx[a];
        for (int a = 0; a < nu; a++) w[a] = orc_np_expf(-(Drows[(i - lo) * N + exp_idx[a]] / rowmax[i]));
        float s = orc_pairwise_f32(w, nu);
        for (int a = 0; a < nu; a++) Vrows[(i - lo) * N + exp_idx[a]] = orc_f2h(w[a] / s);
    }
    free(kr); free(ckr); free(exp_idx); free(w);
}

/* R4 for rows lo..hi (reranking.py:73-78): V [N][N] (all rows), Vq_rows [hi-lo][N]. */
void orc_rr_qe_rows(const int32_t* R, int64_t K, int k2, int64_t lo, int64_t hi, const uint16_t* V, int64_t N,
                    uint16_t* Vq_rows) {
    float* acc = (float*)malloc(sizeof(float) * (size_t)N);
    for (int64_t i = lo; i < hi; i++) {
        for (int64_t c = 0; c < N; c++) acc[c] = 0.0f;
        for (int r = 0; r < k2; r++) {
            const uint16_t* row = V + (int64_t)R[i * K + r] * N;
            for (int64_t c = 0; c < N; c++) acc[c] += orc_h2f(row[c]);
        }
        for (int64_t c = 0; c < N; c++) Vq_rows[(i - lo) * N + c] = orc_f2h(acc[c] / (float)k2);
    }
    free(acc);
}

/* R5-R7 for queries qlo..qhi (reranking.py:80-100): Drows [qhi-qlo][N], rowmax [N],
 * Vq [N][N] (all rows).  out [qhi-qlo][N-Q] float32. */
void orc_rr_jaccard_rows(const float* Drows, const float* rowmax, int64_t Q, int64_t qlo, int64_t qhi,
                         const uint16_t* Vq, int64_t N, uint16_t one_minus_lambda_h, float lambda_f, float* out) {
    int64_t G = N - Q;
    int64_t* cnt = (int64_t*)calloc((size_t)N + 1, sizeof(int64_t));
    for (int64_t r = 0; r < N; r++)
        for (int64_t c = 0; c < N; c++) if (Vq[r * N + c] & 0x7fffu) cnt[c + 1]++;
    for (int64_t c = 0; c < N; c++) cnt[c + 1] += cnt[c];
    int32_t* inv = (int32_t*)malloc(sizeof(int32_t) * (size_t)(cnt[N] > 0 ? cnt[N] : 1));
    int64_t* pos = (int64_t*)malloc(sizeof(int64_t) * (size_t)N);
    for (int64_t c = 0; c < N; c++) pos[c] = cnt[c];
    for (int64_t r = 0; r < N; r++)
        for (int64_t c = 0; c < N; c++) if (Vq[r * N + c] & 0x7fffu) inv[pos[c]++] = (int32_t)r;
    uint16_t* tmin = (uint16_t*)malloc(sizeof(uint16_t) * (size_t)N);
    for (int64_t i = qlo; i < qhi; i++) {
        for (int64_t r = 0; r < N; r++) tmin[r] = 0;
        for (int64_t c = 0; c < N; c++) {
            uint16_t vi = Vq[i * N + c];
            if (!(vi & 0x7fffu)) continue;
            float fvi = orc_h2f(vi);
            for (int64_t p = cnt[c]; p < cnt[c + 1]; p++) {
                int32_t r = inv[p];
                float fvr = orc_h2f(Vq[(int64_t)r * N + c]);
                float mn = fvr < fvi ? fvr : fvi;
                tmin[r] = orc_f2h(orc_h2f(tmin[r]) + mn);
            }
        }
        for (int64_t r = Q; r < N; r++) {
            float t = orc_h2f(tmin[r]);
            uint16_t den = orc_f2h(2.0f - t);
            uint16_t qt = orc_f2h(t / orc_h2f(den));
            uint16_t jac = orc_f2h(1.0f - orc_h2f(qt));
            float a = orc_h2f(orc_f2h(orc_h2f(jac) * orc_h2f(one_minus_lambda_h)));
            float b = (Drows[(i - qlo) * N + r] / rowmax[i]) * lambda_f;
            out[(i - qlo) * G + (r - Q)] = a + b;
        }
    }
    free(cnt); free(inv); free(pos); free(tmin);
}
