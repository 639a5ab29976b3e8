/*
 * asan_driver.c — runs the C restatement (reid_oracle.c, transforms_oracle.c) under
 * AddressSanitizer + UndefinedBehaviorSanitizer ("-fsanitize=address host build
 * of the CPU restatement").  TEST INFRASTRUCTURE ONLY, like the oracle itself.
 *
 * Built by `make -C oracle asan` into build/asan/oracle_asan (a standalone executable: the
 * sanitizer runtime needs no preloading into Python).  tests/test_sanitizers.py writes a batch
 * of calls to stdin, the driver answers on stdout, and the test compares every answer with the
 * same call through the unsanitised liboracle.so (bit for bit) — so the sanitised build runs the
 * oracle tests' own inputs (the golden fixtures' shapes, ties, junk / distractor labels, k1/k2
 * variants) plus edge cases, and any out-of-bounds access, use-after-free, leak or undefined
 * operation aborts the run.
 *
 * Protocol (little-endian): records of  int32 op, int32 nparams, int64 params[nparams], then
 * the op's input arrays (sizes implied by params).  Each answer: the op's output arrays.
 *   op 0 l2norm   (n, d)                     x f32[n*d]                  -> y f32[n*d]
 *   op 1 distmat  (Q, G, D)                  q f32[Q*D], g f32[G*D]      -> f32[Q*G]
 *   op 2 topk     (Q, G, k)                  dist f32[Q*G]               -> i32[Q*k]
 *   op 3 eval     (Q, G)                     dist, qp, gp, qc, gc (i64)  -> valid i32[Q], first i64[Q],
 *                                                                          ap f64[Q], nkept i64[Q]
 *   op 4 rerank   (N, Q, k1, k2, lam_h, lam_f bits)  D f32[N*N]          -> final f32[Q*(N-Q)],
 *                                                                          rank i32[N*K], vqe u16[N*N], jac u16[Q*N]
 *   op 5 resize   (h, w, oh, ow)             img u8[h*w*3]               -> u8[oh*ow*3]
 *   op 6 totensor (h, w)                     img u8[h*w*3], mean f32[3], std f32[3] -> f32[3*h*w]
 *   op 7 threads  (n)                                                    -> (nothing)
 *   op -1 end
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

void orc_set_threads(int n);
void orc_l2norm(const float* x, float* y, int64_t n, int64_t d);
void orc_distmat(const float* q, const float* g, int64_t Q, int64_t G, int64_t D, float* out);
void orc_topk_rows(const float* dist, int64_t Q, int64_t G, int64_t k, int32_t* out);
void orc_eval_rows(const float* dist, int64_t Q, int64_t G, const int64_t* qp, const int64_t* gp, const int64_t* qc,
                   const int64_t* gc, int32_t* valid, int64_t* first, double* ap, int64_t* nkept);
int orc_rerank_from_dist(const float* D, int64_t N, int64_t Q, int k1, int k2, uint16_t one_minus_lambda_h,
                         float lambda_f, float* final_out, int32_t* rank_out, uint16_t* vqe_out, uint16_t* jac_out);
void orc_pil_resize_rgb(const uint8_t* src, int h, int w, int oh, int ow, uint8_t* dst);
void orc_to_tensor_normalize(const uint8_t* hwc, int h, int w, const float* mean, const float* std, float* chw);

static void die(const char* m) {
    fprintf(stderr, "asan_driver: %s\n", m);
    exit(2);
}

/* exactly-sized heap buffers, so ASan sees any access past a buffer the caller passed */
static void* rd(size_t bytes) {
    void* p = malloc(bytes ? bytes : 1);
    if (!p) die("out of memory");
    if (bytes && fread(p, 1, bytes, stdin) != bytes) die("short input");
    return p;
}

static void* buf(size_t bytes) {
    void* p = malloc(bytes ? bytes : 1);
    if (!p) die("out of memory");
    return p;
}

static void wr(const void* p, size_t bytes) {
    if (bytes && fwrite(p, 1, bytes, stdout) != bytes) die("short output");
}

int main(void) {
    for (;;) {
        int32_t op, np;
        if (fread(&op, 4, 1, stdin) != 1) die("no op");
        if (op < 0) break;
        if (fread(&np, 4, 1, stdin) != 1 || np < 0 || np > 8) die("bad param count");
        int64_t p[8] = {0};
        if (np && fread(p, 8, (size_t)np, stdin) != (size_t)np) die("short params");
        if (op == 0) {
            const size_t n = (size_t)(p[0] * p[1]);
            float* x = rd(4 * n);
            float* y = buf(4 * n);
            orc_l2norm(x, y, p[0], p[1]);
            wr(y, 4 * n);
            free(x);
            free(y);
        } else if (op == 1) {
            float* q = rd(4 * (size_t)(p[0] * p[2]));
            float* g = rd(4 * (size_t)(p[1] * p[2]));
            float* o = buf(4 * (size_t)(p[0] * p[1]));
            orc_distmat(q, g, p[0], p[1], p[2], o);
            wr(o, 4 * (size_t)(p[0] * p[1]));
            free(q);
            free(g);
            free(o);
        } else if (op == 2) {
            float* d = rd(4 * (size_t)(p[0] * p[1]));
            int32_t* o = buf(4 * (size_t)(p[0] * p[2]));
            orc_topk_rows(d, p[0], p[1], p[2], o);
            wr(o, 4 * (size_t)(p[0] * p[2]));
            free(d);
            free(o);
        } else if (op == 3) {
            const int64_t Q = p[0], G = p[1];
            float* d = rd(4 * (size_t)(Q * G));
            int64_t* qp = rd(8 * (size_t)Q);
            int64_t* gp = rd(8 * (size_t)G);
            int64_t* qc = rd(8 * (size_t)Q);
            int64_t* gc = rd(8 * (size_t)G);
            int32_t* valid = buf(4 * (size_t)Q);
            int64_t* first = buf(8 * (size_t)Q);
            double* ap = buf(8 * (size_t)Q);
            int64_t* nkept = buf(8 * (size_t)Q);
            orc_eval_rows(d, Q, G, qp, gp, qc, gc, valid, first, ap, nkept);
            wr(valid, 4 * (size_t)Q);
            wr(first, 8 * (size_t)Q);
            wr(ap, 8 * (size_t)Q);
            wr(nkept, 8 * (size_t)Q);
            free(d);
            free(qp);
            free(gp);
            free(qc);
            free(gc);
            free(valid);
            free(first);
            free(ap);
            free(nkept);
        } else if (op == 4) {
            const int64_t N = p[0], Q = p[1];
            const int k1 = (int)p[2], k2 = (int)p[3];
            const uint16_t lam_h = (uint16_t)p[4];
            const uint32_t lf_bits = (uint32_t)p[5];
            float lam_f;
            memcpy(&lam_f, &lf_bits, 4);
            int64_t K = k1 + 1 > k2 ? k1 + 1 : k2;
            if (K > N) K = N;
            float* D = rd(4 * (size_t)(N * N));
            float* fin = buf(4 * (size_t)(Q * (N - Q)));
            int32_t* rank = buf(4 * (size_t)(N * K));
            uint16_t* vqe = buf(2 * (size_t)(N * N));
            uint16_t* jac = buf(2 * (size_t)(Q * N));
            orc_rerank_from_dist(D, N, Q, k1, k2, lam_h, lam_f, fin, rank, vqe, jac);
            wr(fin, 4 * (size_t)(Q * (N - Q)));
            wr(rank, 4 * (size_t)(N * K));
            wr(vqe, 2 * (size_t)(N * N));
            wr(jac, 2 * (size_t)(Q * N));
            free(D);
            free(fin);
            free(rank);
            free(vqe);
            free(jac);
        } else if (op == 5) {
            const int h = (int)p[0], w = (int)p[1], oh = (int)p[2], ow = (int)p[3];
            uint8_t* img = rd((size_t)h * w * 3);
            uint8_t* o = buf((size_t)oh * ow * 3);
            orc_pil_resize_rgb(img, h, w, oh, ow, o);
            wr(o, (size_t)oh * ow * 3);
            free(img);
            free(o);
        } else if (op == 6) {
            const int h = (int)p[0], w = (int)p[1];
            uint8_t* img = rd((size_t)h * w * 3);
            float* mean = rd(12);
            float* std = rd(12);
            float* o = buf(4 * (size_t)3 * h * w);
            orc_to_tensor_normalize(img, h, w, mean, std, o);
            wr(o, 4 * (size_t)3 * h * w);
            free(img);
            free(mean);
            free(std);
            free(o);
        } else if (op == 7) {
            orc_set_threads((int)p[0]);
        } else {
            die("unknown op");
        }
    }
    fflush(stdout);
    return 0;
}
