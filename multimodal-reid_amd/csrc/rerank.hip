// rerank.hip — k-reciprocal re-ranking (reranking.py:29-100, Zhong et al. CVPR'17) on gfx950.
//
// Stage map, all bit-exact with oracle/reid_oracle.c:
//   R1 distmat over cat(q, g)                    backend.hip distmat (exact fp32)      reranking.py:36-41
//   R2 od = D / colmax, initial_rank[:, :K]      rowmax + topk (stable ties)           reranking.py:45-48
//   R3 k-reciprocal expansion + V row            kreciprocal_kernel  (ELL, fp16)       reranking.py:51-71
//   R4 query expansion V_qe = mean of k2 rows    qe_kernel            (ELL, fp16)      reranking.py:73-78
//   R5 inverted index                            csc_count/scan/fill  (CSC)            reranking.py:80-82
//   R6+R7 Jaccard with sequential fp16 sums, blend with od, slice [:Q, Q:]  jaccard_kernel  reranking.py:84-100
// The reference keeps V, V_qe as dense N x N fp16 (2 x 35 GB at MSMT17) and loops in Python;
// here V/V_qe are row-sorted ELL (column index + fp16 bits) and the inverted index is CSC,
// so memory is O(N * nnz) and every stage is a data-parallel kernel.
// Arithmetic mirrors numpy exactly: float32 exp = numpy's AVX512F/AVX2 polynomial
// (pinned against numpy 2.2.6), float32 pairwise sum, fp16 ufuncs = op in fp32 then RNE.
#include "common.h"

namespace reidmi {

int topk_launch(const float* x, int64_t rows, int64_t cols, int64_t ldx, const float* row_div, int k,
                int32_t* out_idx, float* out_val, int64_t ldo, hipStream_t s);
int distmat_launch(const float* q, int64_t Q, int64_t ldq, const float* g, int64_t G, int64_t ldg, int64_t D,
                   float* out, int64_t ldo, float* ws, hipStream_t s);

constexpr int VCAP = 1408;   // >= (k1+1) + (k1+1)(round(k1/2)+1) unique entries for k1 <= 50
constexpr int QCAP = 4096;   // V_qe row capacity
constexpr int LCAP = 6144;   // staged entries of the k2 rows in qe_kernel
constexpr int JCH = 32768;   // gallery columns per Jaccard workgroup (fp16 accumulators in LDS)

enum RrFlag : int { RR_VCAP = 1, RR_QCAP = 2, RR_LCAP = 4 };

// numpy float32 exp (simd_exp_f32, AVX512F/AVX2): see oracle/reid_oracle.c orc_np_expf.
__device__ __forceinline__ float np_expf(float x) {
    if (x != x) return x;
    if (x > 88.72283935546875f) return __builtin_inff();
    if (x < -103.97208404541015625f) return 0.0f;
    const float quad = __builtin_rintf(x * 1.442695040888963407359924681001892137f);
    float r = __builtin_fmaf(quad, -6.93145752e-1f, x);
    r = __builtin_fmaf(quad, -1.42860677e-6f, r);
    float num = __builtin_fmaf(5.082762527590693718096e-04f, r, 6.757896990527504603057e-03f);
    num = __builtin_fmaf(num, r, 5.114512081637298353406e-02f);
    num = __builtin_fmaf(num, r, 2.473615434895520810817e-01f);
    num = __builtin_fmaf(num, r, 7.257664613233124478488e-01f);
    num = __builtin_fmaf(num, r, 9.999999999980870924916e-01f);
    float den = __builtin_fmaf(2.159509375685829852307e-02f, r, -2.742335390411667452936e-01f);
    den = __builtin_fmaf(den, r, 1.0f);
    return __builtin_ldexpf(num / den, (int)quad);
}

// numpy float32 pairwise sum of a[0..n) (PW_BLOCKSIZE 128, 8 accumulators), iterative.
__device__ float pairwise_f32(const float* a, int n) {
    struct F { int off, n, n2, stage; float left; };
    F st[32];
    int sp = 0;
    st[sp++] = F{0, n, 0, 0, 0.f};
    float ret = 0.f;
    while (sp > 0) {
        F& f = st[sp - 1];
        if (f.stage == 0) {
            if (f.n < 8) {
                float res = 0.f;
                for (int i = 0; i < f.n; i++) res += a[f.off + i];
                ret = res; sp--; continue;
            }
            if (f.n <= 128) {
                float r[8];
                for (int j = 0; j < 8; j++) r[j] = a[f.off + j];
                int i;
                for (i = 8; i < f.n - (f.n % 8); i += 8)
                    for (int j = 0; j < 8; j++) r[j] += a[f.off + i + j];
                float res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
                for (; i < f.n; i++) res += a[f.off + i];
                ret = res; sp--; continue;
            }
            int n2 = f.n / 2;
            n2 -= n2 % 8;
            f.n2 = n2;
            f.stage = 1;
            F c{f.off, n2, 0, 0, 0.f};
            st[sp++] = c;
        } else if (f.stage == 1) {
            f.left = ret;
            f.stage = 2;
            F c{f.off + f.n2, f.n - f.n2, 0, 0, 0.f};
            st[sp++] = c;
        } else {
            ret = f.left + ret;
            sp--;
        }
    }
    return ret;
}

// ------------------------------------------------------------------ R2 helpers
__global__ void rowmax_kernel(const float* __restrict__ D, int64_t N, int64_t ld, float* __restrict__ out) {
    const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= N) return;
    const int lane = threadIdx.x & 63;
    float m = -__builtin_inff();
    for (int64_t j = lane; j < N; j += 64) m = fmaxf(m, D[r * ld + j]);
    m = wave_max(m);
    if (lane == 0) out[r] = m;
}

// T = (D + add)^T (a non-symmetric distance: od rows are D columns, reranking.py:46)
__global__ void transpose_kernel(const float* __restrict__ D, const float* __restrict__ add, int64_t N,
                                 float* __restrict__ T) {
    __shared__ float tile[32][33];
    const int64_t bx = (int64_t)blockIdx.x * 32, by = (int64_t)blockIdx.y * 32;
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 256 threads: 32 x 8
    for (int k = ty; k < 32; k += 8) {
        const int64_t r = by + k, c = bx + tx;
        if (r < N && c < N) tile[k][tx] = add ? D[r * N + c] + add[r * N + c] : D[r * N + c];
    }
    __syncthreads();
    for (int k = ty; k < 32; k += 8) {
        const int64_t r = bx + k, c = by + tx;
        if (r < N && c < N) T[r * N + c] = tile[tx][k];
    }
}


// ---------------------------------------------------------------- R3: V rows
__device__ __forceinline__ bool row_has(const int32_t* R, int64_t ldr, int32_t row, int kk, int32_t v) {
    const int32_t* p = R + (int64_t)row * ldr;
    for (int b = 0; b < kk; b++)
        if (p[b] == v) return true;
    return false;
}

__device__ void bitonic_sort_i32(int32_t* a, int P) {
    for (int k = 2; k <= P; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int t = threadIdx.x; t < P; t += blockDim.x) {
                const int o = t ^ j;
                if (o > t) {
                    const bool up = (t & k) == 0;
                    const int32_t x = a[t], y = a[o];
                    if ((x > y) == up) { a[t] = y; a[o] = x; }
                }
            }
            __syncthreads();
        }
}

__device__ __forceinline__ int pow2_ceil_i(int n) {
    int p = 1;
    while (p < n) p <<= 1;
    return p;
}

// One 256-thread workgroup per row i of od.  R: initial_rank [N][ldr] (stable argsort prefix).
__global__ __launch_bounds__(256) void kreciprocal_kernel(const float* __restrict__ OD, int64_t ld,
                                                          const float* __restrict__ rowdiv, const int32_t* __restrict__ R,
                                                          int64_t ldr, int64_t N, int kf, int kh1,
                                                          int32_t* __restrict__ vcol, uint16_t* __restrict__ vval,
                                                          int32_t* __restrict__ vnnz, int32_t* __restrict__ flags) {
    __shared__ int32_t kr[64];
    __shared__ int32_t lst[2048];
    __shared__ float w[2048];
    __shared__ int s_nk, s_n, s_nu;
    __shared__ float s_sum;
    const int64_t i = blockIdx.x;
    const int tid = threadIdx.x;
    // k-reciprocal set of i at depth k1 (reranking.py:53-56), kept in forward order
    if (tid < 64) {
        const int f = tid;
        bool keep = false;
        int32_t c = -1;
        if (f < kf) {
            c = R[i * ldr + f];
            keep = row_has(R, ldr, c, kf, (int32_t)i);
        }
        const unsigned long long m = __ballot(keep);
        const int pos = __popcll(m & ((1ull << f) - 1ull));
        if (keep) kr[pos] = c;
        if (f == 0) s_nk = __popcll(m);
    }
    __syncthreads();
    const int nk = s_nk;
    for (int t = tid; t < nk; t += blockDim.x) lst[t] = kr[t];
    if (tid == 0) s_n = nk;
    __syncthreads();
    // expansion (reranking.py:57-65): candidate a's half-depth reciprocal set is appended when
    // |set ∩ k_reciprocal| > 2/3 |set|; order is irrelevant (np.unique sorts)
    if (tid < nk) {
        const int32_t a = kr[tid];
        int32_t cset[64];
        int nc = 0;
        for (int f = 0; f < kh1; f++) {
            const int32_t c = R[(int64_t)a * ldr + f];
            if (row_has(R, ldr, c, kh1, a)) cset[nc++] = c;
        }
        int inter = 0;
        for (int b = 0; b < nc; b++)
            for (int c = 0; c < nk; c++)
                if (cset[b] == kr[c]) { inter++; break; }
        if ((double)inter > 2.0 / 3.0 * (double)nc) {
            const int base = atomicAdd(&s_n, nc);
            for (int b = 0; b < nc; b++) lst[base + b] = cset[b];
        }
    }
    __syncthreads();
    const int n = s_n;
    const int P = pow2_ceil_i(n < 2 ? 2 : n);
    for (int t = n + tid; t < P; t += blockDim.x) lst[t] = 0x7fffffff;
    __syncthreads();
    bitonic_sort_i32(lst, P);
    // unique (np.unique) by one thread, weights, pairwise sum
    if (tid == 0) {
        int nu = 0;
        for (int t = 0; t < n; t++)
            if (nu == 0 || lst[t] != lst[nu - 1]) lst[nu++] = lst[t];
        s_nu = nu;
    }
    __syncthreads();
    const int nu = s_nu;
    const float dv = rowdiv[i];
    for (int t = tid; t < nu; t += blockDim.x) w[t] = np_expf(-(OD[i * ld + lst[t]] / dv));
    __syncthreads();
    if (tid == 0) s_sum = pairwise_f32(w, nu);
    __syncthreads();
    if (nu > VCAP) {
        if (tid == 0) { atomicOr(flags, RR_VCAP); vnnz[i] = 0; }
        return;
    }
    const float sum = s_sum;
    for (int t = tid; t < nu; t += blockDim.x) {
        vcol[i * VCAP + t] = lst[t];
        vval[i * VCAP + t] = f2h_bits(w[t] / sum);
    }
    if (tid == 0) vnnz[i] = nu;
}

// --------------------------------------------------------------------- R4: QE
// V_qe[i] = fp16( (sum_{j<k2, in order} fp32(V[R[i][j]])) / k2 ) over the union of columns.
// Entries of the k2 (column-sorted) rows are staged in LDS; the first occurrence of each
// column owns it and sums that column over all k2 rows in j order (binary search).
__global__ __launch_bounds__(256) void qe_kernel(const int32_t* __restrict__ R, int64_t ldr, int k2,
                                                 const int32_t* __restrict__ vcol, const uint16_t* __restrict__ vval,
                                                 const int32_t* __restrict__ vnnz, int32_t* __restrict__ qcol,
                                                 uint16_t* __restrict__ qval, int32_t* __restrict__ qnnz,
                                                 int32_t* __restrict__ flags) {
    __shared__ int32_t scol[LCAP];
    __shared__ uint16_t sval[LCAP];
    __shared__ int soff[33];
    __shared__ int32_t ocol[QCAP];
    __shared__ uint16_t oval[QCAP];
    __shared__ int s_no, s_bad;
    const int64_t i = blockIdx.x;
    const int tid = threadIdx.x;
    if (tid == 0) {
        int o = 0;
        for (int j = 0; j < k2; j++) {
            soff[j] = o;
            o += vnnz[R[i * ldr + j]];
        }
        soff[k2] = o;
        s_no = 0;
        s_bad = o > LCAP;
    }
    __syncthreads();
    if (s_bad) {
        if (tid == 0) { atomicOr(flags, RR_LCAP); qnnz[i] = 0; }
        return;
    }
    for (int j = 0; j < k2; j++) {
        const int64_t r = R[i * ldr + j];
        const int n = soff[j + 1] - soff[j];
        for (int t = tid; t < n; t += blockDim.x) {
            scol[soff[j] + t] = vcol[r * VCAP + t];
            sval[soff[j] + t] = vval[r * VCAP + t];
        }
    }
    __syncthreads();
    const int tot = soff[k2];
    const float fk2 = (float)k2;
    for (int e = tid; e < tot; e += blockDim.x) {
        int j = 0;
        while (soff[j + 1] <= e) j++;
        const int32_t c = scol[e];
        bool first = true;
        float acc = 0.f;
        for (int jj = 0; jj < k2; jj++) {
            int lo = soff[jj], hi = soff[jj + 1];
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (scol[mid] < c) lo = mid + 1; else hi = mid;
            }
            const bool hit = lo < soff[jj + 1] && scol[lo] == c;
            if (hit && jj < j) { first = false; break; }
            if (hit) acc += h2f_bits(sval[lo]);
        }
        if (!first) continue;
        const uint16_t h = f2h_bits(acc / fk2);
        if (h & 0x7fff) {
            const int p = atomicAdd(&s_no, 1);
            if (p < QCAP) { ocol[p] = c; oval[p] = h; }
        }
    }
    __syncthreads();
    const int no = s_no;
    if (no > QCAP) {
        if (tid == 0) { atomicOr(flags, RR_QCAP); qnnz[i] = 0; }
        return;
    }
    // sort (column, bits) pairs by column: reuse the int sort on packed keys
    const int P = pow2_ceil_i(no < 2 ? 2 : no);
    int32_t* keys = scol;  // staged rows no longer needed; LCAP >= QCAP
    __syncthreads();
    for (int t = tid; t < P; t += blockDim.x) keys[t] = t < no ? t : 0x7fffffff;
    __syncthreads();
    // sort indices by ocol (columns are unique): bitonic on (ocol[idx])
    for (int k = 2; k <= P; k <<= 1)
        for (int jst = k >> 1; jst > 0; jst >>= 1) {
            for (int t = tid; t < P; t += blockDim.x) {
                const int o = t ^ jst;
                if (o > t) {
                    const bool up = (t & k) == 0;
                    const int32_t x = keys[t], y = keys[o];
                    const int32_t cx = x == 0x7fffffff ? 0x7fffffff : ocol[x];
                    const int32_t cy = y == 0x7fffffff ? 0x7fffffff : ocol[y];
                    if ((cx > cy) == up) { keys[t] = y; keys[o] = x; }
                }
            }
            __syncthreads();
        }
    for (int t = tid; t < no; t += blockDim.x) {
        const int32_t k = keys[t];
        qcol[i * QCAP + t] = ocol[k];
        qval[i * QCAP + t] = oval[k];
    }
    if (tid == 0) qnnz[i] = no;
}

// ------------------------------------------------------------------ R5: CSC
__global__ void csc_count_kernel(const int32_t* __restrict__ qcol, const int32_t* __restrict__ qnnz, int64_t N,
                                 int32_t* __restrict__ cnt) {
    const int64_t r = blockIdx.x;
    for (int t = threadIdx.x; t < qnnz[r]; t += blockDim.x) atomicAdd(&cnt[qcol[r * QCAP + t]], 1);
}

// exclusive scan of cnt[0..N) into off[0..N] (single workgroup, 1024 threads)
__global__ __launch_bounds__(1024) void scan_kernel(const int32_t* __restrict__ cnt, int64_t N, int64_t* __restrict__ off) {
    __shared__ int64_t part[1024];
    const int64_t per = (N + 1023) / 1024;
    const int64_t lo = threadIdx.x * per, hi = lo + per < N ? lo + per : N;
    int64_t s = 0;
    for (int64_t k = lo; k < hi; k++) s += cnt[k];
    part[threadIdx.x] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        int64_t acc = 0;
        for (int t = 0; t < 1024; t++) { const int64_t v = part[t]; part[t] = acc; acc += v; }
        off[N] = acc;
    }
    __syncthreads();
    int64_t acc = part[threadIdx.x];
    for (int64_t k = lo; k < hi; k++) { off[k] = acc; acc += cnt[k]; }
}

__global__ void csc_fill_kernel(const int32_t* __restrict__ qcol, const uint16_t* __restrict__ qval,
                                const int32_t* __restrict__ qnnz, int64_t N, const int64_t* __restrict__ off,
                                int32_t* __restrict__ cur, int32_t* __restrict__ irow, uint16_t* __restrict__ ival) {
    const int64_t r = blockIdx.x;
    for (int t = threadIdx.x; t < qnnz[r]; t += blockDim.x) {
        const int32_t c = qcol[r * QCAP + t];
        const int64_t p = off[c] + atomicAdd(&cur[c], 1);
        irow[p] = (int32_t)r;
        ival[p] = qval[r * QCAP + t];
    }
}

// ----------------------------------------------------------- R6 + R7: Jaccard
// One workgroup per (query i, chunk of gallery columns).  temp_min[r] (fp16 bits) lives in
// LDS; the nonzero columns c of V_qe[i] are visited in ascending order and each column's
// inverted list updates distinct rows, so one barrier per column keeps every temp_min[r]
// a sequential fp16 sum in ascending c (reranking.py:90-92).  Epilogue: Jaccard in fp16
// (reranking.py:93), blend with od in fp32 (reranking.py:95), write final[i][r-Q].
__global__ __launch_bounds__(256) void jaccard_kernel(const float* __restrict__ OD, int64_t ld,
                                                      const float* __restrict__ rowdiv, int64_t Q, int64_t N,
                                                      const int32_t* __restrict__ qcol, const uint16_t* __restrict__ qval,
                                                      const int32_t* __restrict__ qnnz, const int64_t* __restrict__ off,
                                                      const int32_t* __restrict__ irow, const uint16_t* __restrict__ ival,
                                                      uint16_t lam16, float lam_f, float* __restrict__ out, int64_t ldo) {
    __shared__ uint16_t tmin[JCH];
    const int64_t i = blockIdx.y;
    const int64_t base = Q + (int64_t)blockIdx.x * JCH;
    const int64_t end = base + JCH < N ? base + JCH : N;
    const int span = (int)(end - base);
    for (int t = threadIdx.x; t < span; t += blockDim.x) tmin[t] = 0;
    __syncthreads();
    const int nz = qnnz[i];
    for (int e = 0; e < nz; e++) {
        const int32_t c = qcol[i * QCAP + e];
        const float vi = h2f_bits(qval[i * QCAP + e]);
        const int64_t p0 = off[c], p1 = off[c + 1];
        for (int64_t p = p0 + threadIdx.x; p < p1; p += blockDim.x) {
            const int64_t r = irow[p];
            if (r < base || r >= end) continue;
            const float vr = h2f_bits(ival[p]);
            const float mn = vr < vi ? vr : vi;
            const int k = (int)(r - base);
            tmin[k] = f2h_bits(h2f_bits(tmin[k]) + mn);
        }
        __syncthreads();
    }
    const float lam = h2f_bits(lam16);
    const float dv = rowdiv[i];
    for (int t = threadIdx.x; t < span; t += blockDim.x) {
        const int64_t r = base + t;
        const float tv = h2f_bits(tmin[t]);
        const uint16_t den = f2h_bits(2.0f - tv);
        const uint16_t qt = f2h_bits(tv / h2f_bits(den));
        const uint16_t jac = f2h_bits(1.0f - h2f_bits(qt));
        const float a = h2f_bits(f2h_bits(h2f_bits(jac) * lam));
        const float b = (OD[i * ld + r] / dv) * lam_f;
        out[i * ldo + (r - Q)] = a + b;
    }
}

// ---------------------------------------------------------------- workspace
struct RrPlan {
    int64_t dist, tdist, rowmax, rank, vcol, vval, vnnz, qcol, qval, qnnz, cnt, off, cur, irow, ival, total;
    int K;
};

static int64_t al(int64_t v) { return (v + 255) & ~(int64_t)255; }

static RrPlan rr_plan(int64_t N, int k1, int k2, bool need_dist, bool need_t) {
    RrPlan p{};
    int K = k1 + 1 > k2 ? k1 + 1 : k2;
    if (K > N) K = (int)N;
    p.K = K;
    int64_t o = 0;
    p.dist = o; o = al(o + (need_dist ? N * N * 4 : 0) + (need_dist ? N * 4 : 0));
    p.tdist = o; o = al(o + (need_t ? N * N * 4 : 0));
    p.rowmax = o; o = al(o + N * 4);
    p.rank = o; o = al(o + N * (int64_t)K * 4);
    p.vcol = o; o = al(o + N * (int64_t)VCAP * 4);
    p.vval = o; o = al(o + N * (int64_t)VCAP * 2);
    p.vnnz = o; o = al(o + N * 4);
    p.qcol = o; o = al(o + N * (int64_t)QCAP * 4);
    p.qval = o; o = al(o + N * (int64_t)QCAP * 2);
    p.qnnz = o; o = al(o + N * 4);
    p.cnt = o; o = al(o + N * 4);
    p.off = o; o = al(o + (N + 1) * 8);
    p.cur = o; o = al(o + N * 4);
    p.irow = o; o = al(o + N * (int64_t)QCAP * 4);
    p.ival = o; o = al(o + N * (int64_t)QCAP * 2);
    p.total = o;
    return p;
}

// od rows: OD (N x N, row i = distances from item i, scaled by 1/rowdiv[i] on the fly).
static int rerank_core(const float* OD, int64_t N, int64_t Q, int k1, int k2, uint16_t lam16, float lam_f,
                       float* out, int64_t ldo, char* ws, const RrPlan& P, int32_t* flags, hipStream_t s) {
    float* rmax = (float*)(ws + P.rowmax);
    int32_t* R = (int32_t*)(ws + P.rank);
    hipLaunchKernelGGL(rowmax_kernel, dim3(ceil_div(N, 4)), dim3(256), 0, s, OD, N, N, rmax);
    RM_LAUNCHED();
    int rc;
    if ((rc = topk_launch(OD, N, N, N, rmax, P.K, R, nullptr, P.K, s))) return rc;
    const int kf = (int)(k1 + 1 < N ? k1 + 1 : N);
    const int kh = (int)__builtin_nearbyint((double)k1 / 2.0);
    const int kh1 = (int)(kh + 1 < N ? kh + 1 : N);
    RM_REQUIRE(k1 >= 1 && k1 <= 50, "rerank: 1 <= k1 <= 50 (expansion list capacity)");
    int32_t* vcol = (int32_t*)(ws + P.vcol);
    uint16_t* vval = (uint16_t*)(ws + P.vval);
    int32_t* vnnz = (int32_t*)(ws + P.vnnz);
    hipLaunchKernelGGL(kreciprocal_kernel, dim3((unsigned)N), dim3(256), 0, s, OD, N, rmax, R, (int64_t)P.K, N, kf,
                       kh1, vcol, vval, vnnz, flags);
    RM_LAUNCHED();
    int32_t* qcol = (int32_t*)(ws + P.qcol);
    uint16_t* qval = (uint16_t*)(ws + P.qval);
    int32_t* qnnz = (int32_t*)(ws + P.qnnz);
    if (k2 != 1) {
        RM_REQUIRE(k2 <= 32 && k2 <= P.K, "rerank: k2 must be <= 32");
        hipLaunchKernelGGL(qe_kernel, dim3((unsigned)N), dim3(256), 0, s, R, (int64_t)P.K, k2, vcol, vval, vnnz, qcol,
                           qval, qnnz, flags);
        RM_LAUNCHED();
    } else {
        RM_CHECK_HIP(hipMemcpy2DAsync(qcol, QCAP * 4, vcol, VCAP * 4, VCAP * 4, N, hipMemcpyDeviceToDevice, s));
        RM_CHECK_HIP(hipMemcpy2DAsync(qval, QCAP * 2, vval, VCAP * 2, VCAP * 2, N, hipMemcpyDeviceToDevice, s));
        RM_CHECK_HIP(hipMemcpyAsync(qnnz, vnnz, N * 4, hipMemcpyDeviceToDevice, s));
    }
    int32_t* cnt = (int32_t*)(ws + P.cnt);
    int64_t* off = (int64_t*)(ws + P.off);
    int32_t* cur = (int32_t*)(ws + P.cur);
    RM_CHECK_HIP(hipMemsetAsync(cnt, 0, N * 4, s));
    RM_CHECK_HIP(hipMemsetAsync(cur, 0, N * 4, s));
    hipLaunchKernelGGL(csc_count_kernel, dim3((unsigned)N), dim3(256), 0, s, qcol, qnnz, N, cnt);
    RM_LAUNCHED();
    hipLaunchKernelGGL(scan_kernel, dim3(1), dim3(1024), 0, s, cnt, N, off);
    RM_LAUNCHED();
    hipLaunchKernelGGL(csc_fill_kernel, dim3((unsigned)N), dim3(256), 0, s, qcol, qval, qnnz, N, off, cur,
                       (int32_t*)(ws + P.irow), (uint16_t*)(ws + P.ival));
    RM_LAUNCHED();
    const int64_t G = N - Q;
    if (Q > 0 && G > 0) {
        dim3 grid(ceil_div(G, JCH), (unsigned)Q);
        hipLaunchKernelGGL(jaccard_kernel, grid, dim3(256), 0, s, OD, N, rmax, Q, N, qcol, qval, qnnz, off,
                           (const int32_t*)(ws + P.irow), (const uint16_t*)(ws + P.ival), lam16, lam_f, out, ldo);
        RM_LAUNCHED();
    }
    return OK;
}

}  // namespace reidmi

using namespace reidmi;

// from_dist = 0: reidmi_rerank (distance computed inside); 1: reidmi_rerank_from_dist with
// need_transpose = (!symmetric || add != NULL).
REIDMI_API int64_t reidmi_rerank_workspace_bytes(int64_t Q, int64_t G, int k1, int k2, int from_dist,
                                                 int need_transpose) {
    const int64_t N = Q + G;
    return rr_plan(N, k1, k2, !from_dist, from_dist && need_transpose).total;
}

REIDMI_API int reidmi_rerank(const float* feat, int64_t Q, int64_t G, int64_t D, int64_t ldf, int k1, int k2,
                             uint16_t one_minus_lambda_h, float lambda_f, float* final_dist, int64_t ldo, void* ws_,
                             int64_t ws_bytes, int32_t* flags, void* stream) {
    const int64_t N = Q + G;
    RM_REQUIRE(Q >= 0 && G >= 0 && N > 0 && D > 0 && ldf >= D && ldo >= G && flags, "rerank: bad arguments");
    RM_REQUIRE(N < 0x7fffffff, "rerank: too many items");
    const RrPlan P = rr_plan(N, k1, k2, true, false);
    RM_REQUIRE(ws_bytes >= P.total, "rerank: workspace too small");
    hipStream_t s = (hipStream_t)stream;
    char* ws = (char*)ws_;
    float* Dm = (float*)(ws + P.dist);
    int rc;
    // R1: exact-fp32 distance over cat(q, g); symmetric bit-for-bit, so od rows = D rows
    if ((rc = distmat_launch(feat, N, ldf, feat, N, ldf, D, Dm, N, Dm + N * N, s))) return rc;
    return rerank_core(Dm, N, Q, k1, k2, one_minus_lambda_h, lambda_f, final_dist, ldo, ws, P, flags, s);
}

REIDMI_API int reidmi_rerank_from_dist(const float* dist, const float* add, int64_t Q, int64_t G, int symmetric,
                                       int k1, int k2, uint16_t one_minus_lambda_h, float lambda_f, float* final_dist,
                                       int64_t ldo, void* ws_, int64_t ws_bytes, int32_t* flags, void* stream) {
    const int64_t N = Q + G;
    RM_REQUIRE(Q >= 0 && G >= 0 && N > 0 && ldo >= G && flags, "rerank_from_dist: bad arguments");
    const bool need_t = !symmetric || add != nullptr;
    const RrPlan P = rr_plan(N, k1, k2, false, need_t);
    RM_REQUIRE(ws_bytes >= P.total, "rerank_from_dist: workspace too small");
    hipStream_t s = (hipStream_t)stream;
    char* ws = (char*)ws_;
    const float* OD = dist;
    if (need_t) {
        float* T = (float*)(ws + P.tdist);
        hipLaunchKernelGGL(transpose_kernel, dim3(ceil_div(N, 32), ceil_div(N, 32)), dim3(256), 0, s, dist, add, N, T);
        RM_LAUNCHED();
        OD = T;
    }
    return rerank_core(OD, N, Q, k1, k2, one_minus_lambda_h, lambda_f, final_dist, ldo, ws, P, flags, s);
}
