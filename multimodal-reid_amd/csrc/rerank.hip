// rerank.hip — k-reciprocal re-ranking (reranking.py:29-100, Zhong et al. CVPR'17) on gfx950.
//
// Stage map, all bit-exact with oracle/reid_oracle.c:
//   R1 distmat over cat(q, g)                    backend.hip distmat (exact fp32)      reranking.py:36-41
//   R2 od = D / colmax, initial_rank[:, :K]      rowmax + topk (stable ties)           reranking.py:45-48
//   R3 k-reciprocal expansion + V row            kreciprocal_kernel  (ELL, fp16)       reranking.py:51-71
//   R4 query expansion V_qe = mean of k2 rows    qe_kernel            (ELL, fp16)      reranking.py:73-78
//   R5 inverted index                            csc_count/scan/fill(/sort) (CSC)      reranking.py:80-82
//   R6+R7 Jaccard with sequential fp16 sums, blend with od, slice [:Q, Q:]  jaccard_kernel  reranking.py:84-100
// Two drivers: one-call (reidmi_rerank*: N x N distance materialised, capacity-sized ELL
// rows) and staged (reidmi_rr_*: row ranges over exactly sized CSR buffers, distance rows
// in chunks or recomputed, shardable over ranks; see multimodal_reid_amd/reranking.py).
// The reference keeps V, V_qe as dense N x N fp16 (2 x 35 GB at MSMT17) and loops in Python;
// here V/V_qe are row-sorted ELL (column index + fp16 bits) and the inverted index is CSC,
// so memory is O(N * nnz) and every stage is a data-parallel kernel.
// Arithmetic mirrors numpy exactly: float32 exp = numpy's AVX512F/AVX2 polynomial
// (pinned against numpy 2.2.6), float32 pairwise sum, fp16 ufuncs = op in fp32 then RNE.
#include <algorithm>
#include "common.h"
#include "gemm.h"


namespace reidmi {

int rank_select_launch(float* dot, int64_t ldd, const float* feat, int64_t ldf, int D, const float* sqn,
                       const float* nrm, const float* nmax2, int64_t row0, int64_t rows, int64_t N, int K,
                       int32_t* rank_out, float* rowmax_out, int32_t* need, hipStream_t s);
void rank_select_consts(int D, float c[3]);
int norm_max_launch(const float* sqn, const float* nrm, int64_t N, float* out2, hipStream_t s);
int rr_sample_launch(const float* hs, int64_t lds, int64_t ns, const float* sqn, const float* nrm, const float* nmax2,
                     int64_t row0, int64_t rows, int K, int D, float4* meta, float* wrow, int32_t* cnt, int cap,
                     hipStream_t s);
int rank_select_sv_launch(const int32_t* cnt, const int2* list, int cap, const float* wrow, const float* feat,
                          int64_t ldf, int D, const float* sqn, int64_t row0, int64_t rows, int K, int32_t* rank_out,
                          float* rowmax_out, int32_t* need, hipStream_t s);
int feat16_launch(const float* x, int64_t N, int64_t D, int64_t ldx, void* y, int64_t Np, int64_t Dp,
                  int32_t* range_ok, hipStream_t s);
int topk_launch(const float* x, int64_t rows, int64_t cols, int64_t ldx, const float* row_div, int k,
                int32_t* out_idx, float* out_val, int64_t ldo, hipStream_t s);
int distmat_self_launch(const float* x, int64_t N, int64_t ldx, int64_t D, float* out, int64_t ldo, float* ws,
                        hipStream_t s);
int distmat_launch(const float* q, int64_t Q, int64_t ldq, const float* g, int64_t G, int64_t ldg, int64_t D,
                   float* out, int64_t ldo, float* ws, hipStream_t s);
int distmat_pre_launch(const float* q, int64_t Q, int64_t ldq, const float* g, int64_t G, int64_t ldg, int64_t D,
                       const float* qq, const float* gg, float* out, int64_t ldo, hipStream_t s);

// No capacity limits (the reference has none, reranking.py:51-78): every bound below only
// picks the kernel.  A V row holds at most kf (kh1 + 1) entries (the k-reciprocal set plus one
// half-depth set per accepted candidate), so its ELL width is that bound (rr_caps); rows whose
// expansion list fits KR_LST run in LDS (kreciprocal_kernel, k1 <= 61), others on workspace
// scratch (kreciprocal_generic_kernel).  A V_qe row of k2 <= QE_FAST_K2 rows with at most LCAP
// staged entries and QCAP outputs is assembled in LDS (qe_kernel); any other row is deferred to
// qe_generic_kernel, whose scratch is sized for the worst case (k2 rows of the V bound).
constexpr int KR_LST = 2048;   // expansion list of kreciprocal_kernel (LDS)
constexpr int QCAP = 4096;     // V_qe entries qe_kernel assembles in LDS
constexpr int LCAP = 6144;     // staged entries of the k2 rows in qe_kernel
constexpr int QE_FAST_K2 = 32;
constexpr int GEN_WG = 256;    // workgroups of the generic kernels (one per CU), each with its slab
#ifndef RR_JCH
#define RR_JCH 8192
#endif
constexpr int JCH = RR_JCH;   // gallery columns per Jaccard workgroup (fp16 accumulators in LDS)

// flags: a generic kernel found a row beyond the scratch bound it was sized for (cannot happen
// for bounds from rr_caps; a caller passing smaller scratch gets this instead of a fault)
enum RrFlag : int { RR_SCRATCH = 8 };

static int pow2_ceil64(int64_t n) {
    int64_t p = 2;
    while (p < n) p <<= 1;
    return (int)p;
}
static int64_t al16(int64_t v) { return (v + 15) & ~(int64_t)15; }

// kf = min(k1 + 1, N), kh1 = min(round(k1 / 2) + 1, N): the two depths of reranking.py:53,60
static void kr_depths(int k1, int64_t N, int& kf, int& kh1) {
    kf = (int)(k1 + 1 < N ? k1 + 1 : N);
    const int kh = (int)__builtin_nearbyint((double)k1 / 2.0);  // int(np.around(k1/2))
    kh1 = (int)(kh + 1 < N ? kh + 1 : N);
}

struct RrCaps {
    int kf, kh1, K, k2e;
    int64_t vcap;  // entries of a V row (ELL width)
    int64_t tcap;  // staged entries of a V_qe row: k2e V rows
    int64_t qcap;  // entries of a V_qe row (one-call ELL width)
    bool kr_fast;
};
static RrCaps rr_caps(int64_t N, int k1, int k2) {
    RrCaps c{};
    kr_depths(k1, N, c.kf, c.kh1);
    int64_t K = k1 + 1 > k2 ? k1 + 1 : k2;
    c.K = (int)(K < N ? K : N);
    c.k2e = k2 < c.K ? k2 : c.K;  // initial_rank[i, :k2] has min(k2, N) entries
    const int64_t vb = (int64_t)c.kf * (c.kh1 + 1);
    c.vcap = vb < N ? vb : N;
    c.tcap = (int64_t)c.k2e * c.vcap;
    c.qcap = c.tcap < N ? c.tcap : N;
    c.kr_fast = c.kf <= 64 && c.kh1 <= 32 && vb <= KR_LST;  // (kreciprocal_kernel's masks)
    return c;
}

// Per-workgroup scratch of kreciprocal_generic_kernel (byte offsets in one slab)
struct KrSlab {
    int64_t kr, krs, ncnt, acc, cs, lst, w, bytes;
};
static KrSlab kr_slab(int kf, int kh1) {
    KrSlab s{};
    const int64_t nb = (int64_t)kf * (kh1 + 1);
    int64_t o = 0;
    s.kr = o; o = al16(o + (int64_t)kf * 4);
    s.krs = o; o = al16(o + (int64_t)pow2_ceil64(kf) * 4);
    s.ncnt = o; o = al16(o + (int64_t)kf * 4);
    s.acc = o; o = al16(o + (int64_t)kf * 4);
    s.cs = o; o = al16(o + (int64_t)kf * kh1 * 4);
    s.lst = o; o = al16(o + (int64_t)pow2_ceil64(nb) * 4);
    s.w = o; o = al16(o + nb * 4);
    s.bytes = o;
    return s;
}
// ... and of qe_generic_kernel
struct QeSlab {
    int64_t soff, scol, sval, okey, oval, bytes;
};
static QeSlab qe_slab(int k2e, int64_t tcap) {
    QeSlab s{};
    const int64_t P = pow2_ceil64(tcap);
    int64_t o = 0;
    s.soff = o; o = al16(o + (int64_t)(k2e + 1) * 4);
    s.scol = o; o = al16(o + tcap * 4);
    s.sval = o; o = al16(o + tcap * 2);
    s.okey = o; o = al16(o + P * 4);
    s.oval = o; o = al16(o + P * 2);
    s.bytes = o;
    return s;
}

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

// ------------------------------------------------------------------ row views
// A set of sparse rows: CSR (off != nullptr: row r = [off[r], off[r+1])) or fixed-capacity
// ELL (off == nullptr: row r = [r*cap, r*cap + nnz[r])).  Columns ascending in every row.
struct Rows {
    const int64_t* off;
    const int32_t* nnz;
    int64_t cap;
    const int32_t* col;
    const uint16_t* val;
    __device__ __forceinline__ int64_t beg(int64_t r) const { return off ? off[r] : r * cap; }
    __device__ __forceinline__ int len(int64_t r) const { return (int)(off ? off[r + 1] - off[r] : nnz[r]); }
};

// Where original_dist entries come from: a materialised matrix (od != nullptr: entry
// (i, c) = od[(i - row0) * ld + c]) or recomputed from the features with the distance
// kernel's exact arithmetic — an fmaf chain over k ascending, then fmaf(-2, dot, |i|^2 +
// |c|^2) (backend.hip distmat_f32_kernel; the fp32 MFMA accumulates in the same order).
#ifndef DA_UNROLL
#define DA_UNROLL 16
#endif
struct DistSrc {
    const float* od;
    int64_t ld, row0;
    const float* feat;
    int64_t ldf;
    int D;
    const float* sqn;
};

__device__ __forceinline__ float dist_at(const DistSrc& s, int64_t i, int64_t c) {
    if (s.od) return s.od[(i - s.row0) * s.ld + c];
    const float* a = s.feat + i * s.ldf;
    const float* b = s.feat + c * s.ldf;
    float acc = 0.0f;
    int k = 0;
    if ((s.ldf & 3) == 0) {
        // unrolled so that many row loads are in flight ahead of the (sequential) fma chain
#pragma unroll DA_UNROLL
        for (; k + 4 <= s.D; k += 4) {
            const float4 x = *(const float4*)(a + k), y = *(const float4*)(b + k);
            acc = __builtin_fmaf(x.x, y.x, acc);
            acc = __builtin_fmaf(x.y, y.y, acc);
            acc = __builtin_fmaf(x.z, y.z, acc);
            acc = __builtin_fmaf(x.w, y.w, acc);
        }
    }
    for (; k < s.D; k++) acc = __builtin_fmaf(a[k], b[k], acc);
    return __builtin_fmaf(-2.0f, acc, s.sqn[i] + s.sqn[c]);
}

// ------------------------------------------------------------------ R2 helpers
__global__ void rowmax_kernel(const float* __restrict__ D, int64_t rows, int64_t cols, int64_t ld,
                              float* __restrict__ out) {
    const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= rows) return;
    const int lane = threadIdx.x & 63;
    float m = -__builtin_inff();
    for (int64_t j = lane; j < cols; j += 64) m = fmaxf(m, D[r * ld + j]);
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

// v in R[row][0, kk): every load issued before any compare (no early exit: the loads of a
// scan are independent, so they share one memory round trip per unrolled group)
__device__ __forceinline__ bool row_has_all(const int32_t* R, int64_t ldr, int32_t row, int kk, int32_t v) {
    const int32_t* p = R + (int64_t)row * ldr;
    bool hit = false;
#pragma unroll 16
    for (int b = 0; b < kk; b++) hit |= p[b] == v;
    return hit;
}

// One 256-thread workgroup per row i = row0 + blockIdx.x of od (output row blockIdx.x).
// R: initial_rank [N][ldr] (stable argsort prefix), rowdiv[N] the od divisors.  kf <= 64,
// kh1 <= 32 (rr_caps kr_fast).  The membership scans are spread over the workgroup: one
// (candidate a, depth f) pair per thread for the expansion's half-depth sets (bit f of a
// per-candidate mask), instead of one thread walking a's 26 x 26 scans one load at a time.
__global__ __launch_bounds__(256) void kreciprocal_kernel(DistSrc ds, const float* __restrict__ rowdiv,
                                                          const int32_t* __restrict__ R, int64_t ldr, int64_t row0,
                                                          int kf, int kh1, int32_t* __restrict__ vcol,
                                                          uint16_t* __restrict__ vval, int32_t* __restrict__ vnnz,
                                                          int64_t vcap, int32_t* __restrict__ flags) {
    __shared__ int32_t kr[64];
    __shared__ int32_t cand[64][32];          // R[a][f] of the k-reciprocal items a
    __shared__ uint32_t mpass[64], minkr[64];  // bit f: a in R[R[a][f]][:kh1]; and R[a][f] in kr
    __shared__ int32_t lst[KR_LST];
    __shared__ float w[KR_LST];
    __shared__ int wsum[4];
    __shared__ int s_nk, s_n, s_nu;
    __shared__ float s_sum;
    const int64_t b = blockIdx.x;
    const int64_t i = row0 + b;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    // k-reciprocal set of i at depth k1 (reranking.py:53-56), kept in forward order
    if (tid < 64) {
        const int f = tid;
        bool keep = false;
        int32_t c = -1;
        if (f < kf) {
            c = R[i * ldr + f];
            keep = row_has_all(R, ldr, c, kf, (int32_t)i);
        }
        const unsigned long long m = __ballot(keep);
        const int pos = __popcll(m & ((1ull << f) - 1ull));
        if (keep) kr[pos] = c;
        if (f == 0) s_nk = __popcll(m);
        mpass[f] = 0;
        minkr[f] = 0;
    }
    __syncthreads();
    const int nk = s_nk;
    for (int t = tid; t < nk; t += blockDim.x) lst[t] = kr[t];
    if (tid == 0) s_n = nk;
    // expansion (reranking.py:57-65): candidate a's half-depth reciprocal set
    // {c = R[a][f], f < kh1 : a in R[c][:kh1]} is appended when more than 2/3 of it lies in the
    // k-reciprocal set; order is irrelevant (np.unique sorts)
    for (int p = tid; p < nk * kh1; p += blockDim.x) {
        const int ai = p / kh1, f = p - ai * kh1;
        const int32_t a = kr[ai];
        const int32_t c = R[(int64_t)a * ldr + f];
        cand[ai][f] = c;
        if (row_has_all(R, ldr, c, kh1, a)) {
            bool in = false;
            for (int q = 0; q < nk; q++) in |= kr[q] == c;
            atomicOr(&mpass[ai], 1u << f);
            if (in) atomicOr(&minkr[ai], 1u << f);
        }
    }
    __syncthreads();
    if (tid < nk) {
        const uint32_t mp = mpass[tid];
        const int nc = __popc(mp), inter = __popc(minkr[tid]);
        if ((double)inter > 2.0 / 3.0 * (double)nc) {
            int q = atomicAdd(&s_n, nc);
            for (int f = 0; f < kh1; f++)
                if ((mp >> f) & 1u) lst[q++] = cand[tid][f];
        }
    }
    __syncthreads();
    const int n = s_n;
    const int P = pow2_ceil_i(n < 2 ? 2 : n);
    for (int t = n + tid; t < P; t += blockDim.x) lst[t] = 0x7fffffff;
    __syncthreads();
    bitonic_sort_i32(lst, P);
    // unique (np.unique): thread t owns a contiguous segment, counts its first occurrences,
    // and writes them at the exclusive prefix of the counts (into w's storage, then back)
    {
        const int seg = (n + 255) >> 8, s0 = tid * seg, s1 = s0 + seg < n ? s0 + seg : n;
        int cnt = 0;
        for (int t = s0; t < s1; t++) cnt += (t == 0 || lst[t] != lst[t - 1]);
        int incl = cnt;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int u = __shfl_up(incl, o, 64);
            if (lane >= o) incl += u;
        }
        if (lane == 63) wsum[wv] = incl;
        __syncthreads();
        int pos = incl - cnt;
        for (int q = 0; q < wv; q++) pos += wsum[q];
        int32_t* u = (int32_t*)w;
        for (int t = s0; t < s1; t++)
            if (t == 0 || lst[t] != lst[t - 1]) u[pos++] = lst[t];
        if (tid == 255) s_nu = pos;  // (the last segment ends the list)
        __syncthreads();
        const int nu0 = s_nu;
        for (int t = tid; t < nu0; t += blockDim.x) lst[t] = u[t];
        __syncthreads();
    }
    const int nu = s_nu;
    const float dv = rowdiv[i];
    for (int t = tid; t < nu; t += blockDim.x) w[t] = np_expf(-(dist_at(ds, i, lst[t]) / dv));
    __syncthreads();
    if (tid == 0) s_sum = pairwise_f32(w, nu);
    __syncthreads();
    if (nu > vcap) {  // cannot happen: nu <= kf (kh1 + 1) = the width rr_caps gives
        if (tid == 0) { atomicOr(flags, RR_SCRATCH); vnnz[b] = 0; }
        return;
    }
    const float sum = s_sum;
    for (int t = tid; t < nu; t += blockDim.x) {
        vcol[b * vcap + t] = lst[t];
        vval[b * vcap + t] = f2h_bits(w[t] / sum);
    }
    if (tid == 0) vnnz[b] = nu;
}

// R3 for any k1: the same steps as kreciprocal_kernel with the lists on a per-workgroup slab
// of global scratch (KrSlab; a workgroup's slab is only touched by its own threads, ordered by
// its barriers).  Rows b = blockIdx.x, + gridDim.x, ... < nrows.
__global__ __launch_bounds__(256) void kreciprocal_generic_kernel(DistSrc ds, const float* __restrict__ rowdiv,
                                                                  const int32_t* __restrict__ R, int64_t ldr,
                                                                  int64_t row0, int64_t nrows, int kf, int kh1,
                                                                  KrSlab sl, char* __restrict__ slab,
                                                                  int32_t* __restrict__ vcol,
                                                                  uint16_t* __restrict__ vval,
                                                                  int32_t* __restrict__ vnnz, int64_t vcap,
                                                                  int32_t* __restrict__ flags) {
    __shared__ int wsum[4];
    __shared__ int s_nk, s_n, s_nu;
    __shared__ float s_sum;
    char* base = slab + (int64_t)blockIdx.x * sl.bytes;
    int32_t* kr = (int32_t*)(base + sl.kr);
    int32_t* krs = (int32_t*)(base + sl.krs);
    int32_t* ncnt = (int32_t*)(base + sl.ncnt);
    int32_t* acc = (int32_t*)(base + sl.acc);
    int32_t* cs = (int32_t*)(base + sl.cs);
    int32_t* lst = (int32_t*)(base + sl.lst);
    float* w = (float*)(base + sl.w);
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    for (int64_t b = blockIdx.x; b < nrows; b += gridDim.x) {
        const int64_t i = row0 + b;
        // k-reciprocal set of i at depth kf in forward order (reranking.py:53-56)
        if (tid == 0) s_nk = 0;
        __syncthreads();
        for (int f0 = 0; f0 < kf; f0 += 256) {
            const int f = f0 + tid;
            bool keep = false;
            int32_t c = -1;
            if (f < kf) {
                c = R[i * ldr + f];
                keep = row_has(R, ldr, c, kf, (int32_t)i);
            }
            const unsigned long long m = __ballot(keep);
            if (lane == 0) wsum[wv] = __popcll(m);
            __syncthreads();
            int before = s_nk;
            for (int q = 0; q < wv; q++) before += wsum[q];
            if (keep) kr[before + __popcll(m & ((1ull << lane) - 1ull))] = c;
            __syncthreads();
            if (tid == 0) s_nk += wsum[0] + wsum[1] + wsum[2] + wsum[3];
            __syncthreads();
        }
        const int nk = s_nk;
        // a sorted copy for the intersection counts (np.intersect1d of unique sets)
        const int Pk = pow2_ceil_i(nk < 2 ? 2 : nk);
        for (int t = tid; t < Pk; t += blockDim.x) krs[t] = t < nk ? kr[t] : 0x7fffffff;
        __syncthreads();
        bitonic_sort_i32(krs, Pk);
        // each candidate's half-depth reciprocal set and the 2/3 overlap rule (reranking.py:57-65)
        for (int t = tid; t < nk; t += blockDim.x) {
            const int32_t a = kr[t];
            int32_t* ct = cs + (int64_t)t * kh1;
            int nc = 0;
            for (int f = 0; f < kh1; f++) {
                const int32_t c = R[(int64_t)a * ldr + f];
                if (row_has(R, ldr, c, kh1, a)) ct[nc++] = c;
            }
            int inter = 0;
            for (int q = 0; q < nc; q++) {
                int lo = 0, hi = nk;
                while (lo < hi) {
                    const int mid = (lo + hi) >> 1;
                    if (krs[mid] < ct[q]) lo = mid + 1; else hi = mid;
                }
                inter += lo < nk && krs[lo] == ct[q];
            }
            ncnt[t] = nc;
            acc[t] = (double)inter > 2.0 / 3.0 * (double)nc;
        }
        if (tid == 0) s_n = nk;
        for (int t = tid; t < nk; t += blockDim.x) lst[t] = kr[t];
        __syncthreads();
        for (int t = tid; t < nk; t += blockDim.x)
            if (acc[t]) {
                const int nc = ncnt[t];
                const int bs = atomicAdd(&s_n, nc);
                for (int q = 0; q < nc; q++) lst[bs + q] = cs[(int64_t)t * kh1 + q];
            }
        __syncthreads();
        const int n = s_n;
        const int P = pow2_ceil_i(n < 2 ? 2 : n);
        for (int t = n + tid; t < P; t += blockDim.x) lst[t] = 0x7fffffff;
        __syncthreads();
        bitonic_sort_i32(lst, P);
        if (tid == 0) {  // np.unique
            int nu = 0;
            for (int t = 0; t < n; t++)
                if (nu == 0 || lst[t] != lst[nu - 1]) lst[nu++] = lst[t];
            s_nu = nu;
        }
        __syncthreads();
        const int nu = s_nu;
        const float dv = rowdiv[i];
        for (int t = tid; t < nu; t += blockDim.x) w[t] = np_expf(-(dist_at(ds, i, lst[t]) / dv));
        __syncthreads();
        if (tid == 0) s_sum = pairwise_f32(w, nu);
        __syncthreads();
        if (nu > vcap) {
            if (tid == 0) { atomicOr(flags, RR_SCRATCH); vnnz[b] = 0; }
        } else {
            const float sum = s_sum;
            for (int t = tid; t < nu; t += blockDim.x) {
                vcol[b * vcap + t] = lst[t];
                vval[b * vcap + t] = f2h_bits(w[t] / sum);
            }
            if (tid == 0) vnnz[b] = nu;
        }
        __syncthreads();  // the slab and the shared counters are reused by the next row
    }
}

// --------------------------------------------------------------------- R4: QE
// V_qe[i] = fp16( (sum_{j<k2, in order} fp32(V[R[i][j]])) / k2 ) over the union of columns,
// i = row0 + blockIdx.x (output row blockIdx.x).  Entries of the k2 (column-sorted) rows
// are staged in LDS; the first occurrence of each column owns it and sums that column over
// all k2 rows in j order (binary search).
// A row whose k2 rows stage more than LCAP entries, or that produces more than QCAP, is appended
// to the deferred list (dlist[atomicAdd(dcount)] = b, qnnz[b] = 0) for qe_generic_kernel.
__global__ __launch_bounds__(256) void qe_kernel(const int32_t* __restrict__ R, int64_t ldr, int k2, int64_t row0,
                                                 Rows V, int32_t* __restrict__ qcol, uint16_t* __restrict__ qval,
                                                 int32_t* __restrict__ qnnz, int64_t qcap,
                                                 int32_t* __restrict__ dlist, int32_t* __restrict__ dcount) {
    __shared__ int32_t scol[LCAP];
    __shared__ uint16_t sval[LCAP];
    __shared__ int soff[33];
    __shared__ int32_t ocol[QCAP];
    __shared__ uint16_t oval[QCAP];
    __shared__ int s_no, s_bad;
    __shared__ int64_t s_rb[32];
    __shared__ int s_len[32];
    const int64_t b = blockIdx.x;
    const int64_t i = row0 + b;
    const int tid = threadIdx.x;
    // the k2 rows' extents in parallel (one thread each), then their offsets
    if (tid < k2) {
        const int64_t r = R[i * ldr + tid];
        s_rb[tid] = V.beg(r);
        s_len[tid] = V.len(r);
    }
    __syncthreads();
    if (tid == 0) {
        int o = 0;
        for (int j = 0; j < k2; j++) {
            soff[j] = o;
            o += s_len[j];
        }
        soff[k2] = o;
        s_no = 0;
        s_bad = o > LCAP;
    }
    __syncthreads();
    if (s_bad) {
        if (tid == 0) { qnnz[b] = 0; dlist[atomicAdd(dcount, 1)] = (int32_t)b; }
        return;
    }
    for (int j = 0; j < k2; j++) {
        const int64_t rb = s_rb[j];
        const int n = soff[j + 1] - soff[j];
        for (int t = tid; t < n; t += blockDim.x) {
            scol[soff[j] + t] = V.col[rb + t];
            sval[soff[j] + t] = V.val[rb + t];
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
        if (tid == 0) { qnnz[b] = 0; dlist[atomicAdd(dcount, 1)] = (int32_t)b; }
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
        qcol[b * qcap + t] = ocol[k];
        qval[b * qcap + t] = oval[k];
    }
    if (tid == 0) qnnz[b] = no;
}

// Every row(s) of i = row0 + b to all deferred rows b = dlist[d], d < *dcount (or all rows b <
// nrows when dlist is null): the same arithmetic as qe_kernel (first occurrence of a column owns
// it and sums it over the k2 rows in j order) with the k2 rows staged on a per-workgroup slab
// (QeSlab, sized for k2 rows of the V bound) and the output sorted there.  mode 0: qnnz[b] = the
// row's entry count only; mode 1: the row to CSR at qoff[b] (qnnz untouched); mode 2: the row
// to ELL row b (width qcap) and qnnz[b].
__device__ void bitonic_sort_i32_u16(int32_t* k, uint16_t* v, int P) {
    for (int kk = 2; kk <= P; kk <<= 1)
        for (int j = kk >> 1; j > 0; j >>= 1) {
            for (int t = threadIdx.x; t < P; t += blockDim.x) {
                const int o = t ^ j;
                if (o > t) {
                    const bool up = (t & kk) == 0;
                    const int32_t x = k[t], y = k[o];
                    if ((x > y) == up) {
                        k[t] = y;
                        k[o] = x;
                        const uint16_t a = v[t];
                        v[t] = v[o];
                        v[o] = a;
                    }
                }
            }
            __syncthreads();
        }
}

__global__ __launch_bounds__(256) void qe_generic_kernel(const int32_t* __restrict__ R, int64_t ldr, int k2,
                                                         int64_t row0, Rows V, const int32_t* __restrict__ dlist,
                                                         const int32_t* __restrict__ dcount, int64_t nrows, int mode,
                                                         int32_t* __restrict__ qcol, uint16_t* __restrict__ qval,
                                                         int32_t* __restrict__ qnnz, int64_t qcap,
                                                         const int64_t* __restrict__ qoff, QeSlab sl,
                                                         char* __restrict__ slab, int64_t tcap,
                                                         int32_t* __restrict__ flags) {
    __shared__ int s_tot, s_no;
    char* base = slab + (int64_t)blockIdx.x * sl.bytes;
    int32_t* soff = (int32_t*)(base + sl.soff);
    int32_t* scol = (int32_t*)(base + sl.scol);
    uint16_t* sval = (uint16_t*)(base + sl.sval);
    int32_t* okey = (int32_t*)(base + sl.okey);
    uint16_t* oval = (uint16_t*)(base + sl.oval);
    const int tid = threadIdx.x;
    const int64_t nd = dcount ? (int64_t)*dcount : nrows;
    const float fk2 = (float)k2;
    for (int64_t d = blockIdx.x; d < nd; d += gridDim.x) {
        const int64_t b = dlist ? dlist[d] : d;
        const int64_t i = row0 + b;
        if (tid == 0) {
            int64_t o = 0;
            for (int j = 0; j < k2; j++) {
                soff[j] = (int32_t)o;
                o += V.len(R[i * ldr + j]);
            }
            soff[k2] = (int32_t)(o < tcap ? o : tcap);
            s_tot = o > tcap ? -1 : (int)o;
            s_no = 0;
        }
        __syncthreads();
        const int tot = s_tot;
        if (tot < 0) {  // beyond the slab (not for tcap from rr_caps)
            if (tid == 0) {
                atomicOr(flags, RR_SCRATCH);
                if (mode != 1) qnnz[b] = 0;
            }
            __syncthreads();
            continue;
        }
        for (int j = 0; j < k2; j++) {
            const int64_t rb = V.beg(R[i * ldr + j]);
            const int n = soff[j + 1] - soff[j];
            for (int t = tid; t < n; t += blockDim.x) {
                scol[soff[j] + t] = V.col[rb + t];
                sval[soff[j] + t] = V.val[rb + t];
            }
        }
        __syncthreads();
        for (int e = tid; e < tot; e += blockDim.x) {
            int lo = 0, hi = k2;  // the row of entry e: the largest j with soff[j] <= e
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (soff[mid] <= e) lo = mid; else hi = mid - 1;
            }
            const int j = lo;
            const int32_t c = scol[e];
            bool first = true;
            float acc = 0.f;
            for (int jj = 0; jj < k2; jj++) {
                int a = soff[jj], z = soff[jj + 1];
                while (a < z) {
                    const int mid = (a + z) >> 1;
                    if (scol[mid] < c) a = mid + 1; else z = mid;
                }
                const bool hit = a < soff[jj + 1] && scol[a] == c;
                if (hit && jj < j) { first = false; break; }
                if (hit) acc += h2f_bits(sval[a]);
            }
            if (!first) continue;
            const uint16_t h = f2h_bits(acc / fk2);
            if (h & 0x7fff) {
                const int p = atomicAdd(&s_no, 1);
                okey[p] = c;
                oval[p] = h;
            }
        }
        __syncthreads();
        const int no = s_no;
        if (mode == 0) {
            if (tid == 0) qnnz[b] = no;
            __syncthreads();
            continue;
        }
        const int P = pow2_ceil_i(no < 2 ? 2 : no);
        for (int t = no + tid; t < P; t += blockDim.x) { okey[t] = 0x7fffffff; oval[t] = 0; }
        __syncthreads();
        bitonic_sort_i32_u16(okey, oval, P);
        if (mode == 1) {
            const int64_t o = qoff[b];
            for (int t = tid; t < no; t += blockDim.x) { qcol[o + t] = okey[t]; qval[o + t] = oval[t]; }
        } else {
            for (int t = tid; t < no; t += blockDim.x) { qcol[b * qcap + t] = okey[t]; qval[b * qcap + t] = oval[t]; }
            if (tid == 0) qnnz[b] = no;
        }
        __syncthreads();
    }
}

// ---------------------------------------------------- ELL -> CSR, row lengths
__global__ void rows_len_kernel(Rows V, int64_t n, int32_t* __restrict__ out) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r < n) out[r] = V.len(r);
}

// exclusive scan of cnt[0..N) into off[0..N] (single workgroup, 1024 threads)
__global__ __launch_bounds__(1024) void scan_kernel(const int32_t* __restrict__ cnt, int64_t N, int64_t* __restrict__ off) {
    __shared__ int64_t part[1024];
    const int64_t per = (N + 1023) / 1024;
    const int64_t lo = threadIdx.x * per < N ? threadIdx.x * per : N;
    const int64_t hi = lo + per < N ? lo + per : N;
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

// copy rows of V into CSR storage at off[] (one workgroup per row)
__global__ void rows_pack_kernel(Rows V, const int64_t* __restrict__ off, int32_t* __restrict__ col,
                                 uint16_t* __restrict__ val) {
    const int64_t r = blockIdx.x;
    const int64_t s = V.beg(r), d = off[r];
    const int n = V.len(r);
    for (int t = threadIdx.x; t < n; t += blockDim.x) {
        col[d + t] = V.col[s + t];
        val[d + t] = V.val[s + t];
    }
}

// ------------------------------------------------------------------ R5: CSC
// invIndex[c] = rows r with V_qe[r, c] != 0 (reranking.py:80-82): per-column counts, an
// exclusive scan, an atomic fill, and (staged driver) a per-column sort by row.
__global__ void csc_count_kernel(Rows V, int64_t N, int32_t* __restrict__ cnt) {
    const int64_t r = blockIdx.x;
    const int64_t s = V.beg(r);
    const int n = V.len(r);
    for (int t = threadIdx.x; t < n; t += blockDim.x) atomicAdd(&cnt[V.col[s + t]], 1);
}

// Unsorted inverted index by atomic fill (the one-call paths: sizes unknown on the host).
__global__ void csc_fill_kernel(Rows V, int64_t N, const int64_t* __restrict__ off, int32_t* __restrict__ cur,
                                int32_t* __restrict__ irow, uint16_t* __restrict__ ival) {
    const int64_t r = blockIdx.x;
    const int64_t s = V.beg(r);
    const int n = V.len(r);
    for (int t = threadIdx.x; t < n; t += blockDim.x) {
        const int32_t c = V.col[s + t];
        const int64_t p = off[c] + atomicAdd(&cur[c], 1);
        irow[p] = (int32_t)r;
        ival[p] = V.val[s + t];
    }
}

// Sort each inverted list by row (reranking.py:80-82 lists rows ascending; the staged
// Jaccard kernel binary-searches a list for a chunk's row range).  One workgroup per column;
// rows are unique within a column, so any sort is the stable one.  Lists of up to
// CSC_LDS entries are bitonic-sorted in LDS; longer ones (hub items in very large galleries)
// in a power-of-two padded slice of a global scratch at 2 * off[c] (>= the padded length,
// since pow2_ceil(len) < 2 len).
constexpr int CSC_LDS = 4096;

__global__ __launch_bounds__(256) void csc_sort_kernel(const int64_t* __restrict__ off, int32_t* __restrict__ irow,
                                                       uint16_t* __restrict__ ival, int32_t* __restrict__ sk,
                                                       uint16_t* __restrict__ sv) {
    __shared__ int32_t lk[CSC_LDS];
    __shared__ uint16_t lv[CSC_LDS];
    const int64_t c = blockIdx.x;
    const int64_t b = off[c];
    const int n = (int)(off[c + 1] - b);
    if (n < 2) return;
    int P = 1;
    while (P < n) P <<= 1;
    const bool in_lds = P <= CSC_LDS;
    int32_t* K = in_lds ? lk : sk + 2 * b;
    uint16_t* V = in_lds ? lv : sv + 2 * b;
    for (int t = threadIdx.x; t < P; t += blockDim.x) {
        K[t] = t < n ? irow[b + t] : 0x7fffffff;
        V[t] = t < n ? ival[b + t] : 0;
    }
    __syncthreads();
    for (int k = 2; k <= P; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int t = threadIdx.x; t < P; t += blockDim.x) {
                const int o = t ^ j;
                if (o > t) {
                    const int32_t a = K[t], d = K[o];
                    if ((d < a) == ((t & k) == 0)) {
                        K[t] = d;
                        K[o] = a;
                        const uint16_t va = V[t];
                        V[t] = V[o];
                        V[o] = va;
                    }
                }
            }
            __syncthreads();
        }
    for (int t = threadIdx.x; t < n; t += blockDim.x) {
        irow[b + t] = K[t];
        ival[b + t] = V[t];
    }
}

// ----------------------------------------------------------- R6 + R7: Jaccard
// One workgroup per (query i = q0 + blockIdx.y, chunk of gallery columns).  temp_min[r]
// (fp16 bits) lives in LDS; the nonzero columns c of V_qe[i] are visited in ascending order
// and each column's inverted list (rows ascending) updates distinct rows, so one barrier per
// column keeps every temp_min[r] a sequential fp16 sum in ascending c (reranking.py:90-92);
// the chunk's sub-range of each list is found by binary search.  Epilogue: Jaccard in fp16
// (reranking.py:93), blend with od in fp32 (reranking.py:95), write final[blockIdx.y][r-Q].
// od of (i, r) = OD[blockIdx.y * ld + (r - odc0)] / rowdiv[i].
// Chunk boundaries of every column's sorted row list, once per call: cbnd[c * (nch + 1) + b]
// = first position p in [off[c], off[c+1]) with irow[p] >= Q + b * JCH (b = nch: off[c+1]).
// jaccard_kernel then reads its slice with two loads instead of two binary searches per
// (query row, column) — those searches were a serial chain of dependent loads.
__global__ __launch_bounds__(256) void jaccard_bounds_kernel(const int64_t* __restrict__ off,
                                                             const int32_t* __restrict__ irow, int64_t N, int64_t Q,
                                                             int nch, int64_t* __restrict__ cbnd) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= N * (nch + 1)) return;
    const int64_t c = t / (nch + 1);
    const int b = (int)(t - c * (nch + 1));
    int64_t lo = off[c], hi = off[c + 1];
    if (b < nch) {
        const int64_t key = Q + (int64_t)b * JCH;
        while (lo < hi) { const int64_t m = (lo + hi) >> 1; if (irow[m] < key) lo = m + 1; else hi = m; }
    } else {
        lo = hi;  // every row index is < N
    }
    cbnd[t] = lo;
}

__global__ __launch_bounds__(256) void jaccard_kernel(const float* __restrict__ OD, int64_t ld, int64_t odc0,
                                                      const float* __restrict__ rowdiv, int64_t q0, int64_t Q,
                                                      int64_t N, Rows Vq, const int64_t* __restrict__ off,
                                                      const int32_t* __restrict__ irow, const uint16_t* __restrict__ ival,
                                                      const int64_t* __restrict__ cbnd, uint16_t lam16, float lam_f,
                                                      float* __restrict__ out, int64_t ldo) {
    __shared__ uint16_t tmin[JCH];
    const int64_t y = blockIdx.y;
    const int64_t i = q0 + y;
    const int64_t base = Q + (int64_t)blockIdx.x * JCH;
    const int64_t end = base + JCH < N ? base + JCH : N;
    const int span = (int)(end - base);
    for (int t = threadIdx.x; t < span; t += blockDim.x) tmin[t] = 0;
    __syncthreads();
    const int nz = Vq.len(i);
    const int64_t qb = Vq.beg(i);
    const int nb1 = (int)gridDim.x + 1;
    // V_qe[i]'s columns in batches of 256: each thread fetches one column's value and slice
    // bounds (jaccard_bounds_kernel) at once, so the column walk below has no dependent
    // bound loads; a thread's element of the next column's slice is loaded before the
    // barrier of the current one
    __shared__ int64_t s_p0[256];
    __shared__ int s_n[256];
    __shared__ float s_vi[256];
    for (int e0 = 0; e0 < nz; e0 += 256) {
        const int m = nz - e0 < 256 ? nz - e0 : 256;
        if ((int)threadIdx.x < m) {
            const int32_t c = Vq.col[qb + e0 + threadIdx.x];
            const int64_t p0 = cbnd[(int64_t)c * nb1 + blockIdx.x], p1 = cbnd[(int64_t)c * nb1 + blockIdx.x + 1];
            s_p0[threadIdx.x] = p0;
            s_n[threadIdx.x] = (int)(p1 - p0);
            s_vi[threadIdx.x] = h2f_bits(Vq.val[qb + e0 + threadIdx.x]);
        }
        __syncthreads();
        int nk = -1;
        float nv = 0.0f;
        auto fetch = [&](int e) {
            nk = -1;
            if ((int)threadIdx.x < s_n[e]) {
                const int64_t p = s_p0[e] + threadIdx.x;
                nk = (int)(irow[p] - base);
                nv = h2f_bits(ival[p]);
            }
        };
        fetch(0);
        for (int e = 0; e < m; e++) {
            const int k = nk;
            const float vr = nv;
            const float vi = s_vi[e];
            const int n = s_n[e];
            if (e + 1 < m) fetch(e + 1);
            if (k >= 0) {
                const float mn = vr < vi ? vr : vi;
                tmin[k] = f2h_bits(h2f_bits(tmin[k]) + mn);
            }
            for (int64_t p = s_p0[e] + 256 + threadIdx.x; p < s_p0[e] + n; p += blockDim.x) {  // long slices
                const int kk = (int)(irow[p] - base);
                const float vr2 = h2f_bits(ival[p]);
                const float mn = vr2 < vi ? vr2 : vi;
                tmin[kk] = f2h_bits(h2f_bits(tmin[kk]) + mn);
            }
            __syncthreads();
        }
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
        const float b = (OD[y * ld + (r - odc0)] / dv) * lam_f;
        out[y * ldo + (r - Q)] = a + b;
    }
}

// ---------------------------------------------------------------- workspace
struct RrPlan {
    int64_t dist, tdist, rowmax, rank, vcol, vval, vnnz, qcol, qval, qnnz, cnt, off, cur, irow, ival, dlist, dcount,
        krslab, qeslab, total;
    RrCaps caps;
    KrSlab kr;
    QeSlab qe;
};

static int64_t al(int64_t v) { return (v + 255) & ~(int64_t)255; }

// One-call driver: V and V_qe as ELL of their worst-case widths (rr_caps), so no row can
// overflow; the generic kernels' slabs only when a row can need them.
static RrPlan rr_plan(int64_t N, int k1, int k2, bool need_dist, bool need_t) {
    RrPlan p{};
    p.caps = rr_caps(N, k1, k2);
    const RrCaps& c = p.caps;
    const int64_t qw = k2 != 1 ? c.qcap : 0;
    p.kr = kr_slab(c.kf, c.kh1);
    p.qe = qe_slab(c.k2e, c.tcap);
    int64_t o = 0;
    p.dist = o; o = al(o + (need_dist ? N * N * 4 : 0) + (need_dist ? N * 4 : 0));
    p.tdist = o; o = al(o + (need_t ? N * N * 4 : 0));
    p.rowmax = o; o = al(o + N * 4);
    p.rank = o; o = al(o + N * (int64_t)c.K * 4);
    p.vcol = o; o = al(o + N * c.vcap * 4);
    p.vval = o; o = al(o + N * c.vcap * 2);
    p.vnnz = o; o = al(o + N * 4);
    p.qcol = o; o = al(o + N * qw * 4);
    p.qval = o; o = al(o + N * qw * 2);
    p.qnnz = o; o = al(o + N * 4);
    p.cnt = o; o = al(o + N * 4);
    p.off = o; o = al(o + (N + 1) * 8);
    p.cur = o; o = al(o + N * 4);
    const int64_t inv = k2 != 1 ? qw : c.vcap;  // inverted-index entries per row (upper bound)
    p.irow = o; o = al(o + N * inv * 4);
    p.ival = o; o = al(o + N * inv * 2);
    p.dlist = o; o = al(o + N * 4);
    p.dcount = o; o = al(o + 16);
    p.krslab = o; o = al(o + (c.kr_fast ? 0 : GEN_WG * p.kr.bytes));
    p.qeslab = o; o = al(o + (k2 != 1 ? GEN_WG * p.qe.bytes : 0));
    p.total = o;
    return p;
}

// R3 over rows [row0, row0 + n) into the ELL (vcol, vval, vnnz) of width caps.vcap.
static int v_rows_launch(const DistSrc& ds, const float* rowdiv, const int32_t* R, int64_t ldr, int64_t row0,
                         int64_t n, const RrCaps& c, char* krslab, int32_t* vcol, uint16_t* vval, int32_t* vnnz,
                         int32_t* flags, hipStream_t s) {
    if (n == 0) return OK;
    if (c.kr_fast) {
        hipLaunchKernelGGL(kreciprocal_kernel, dim3((unsigned)n), dim3(256), 0, s, ds, rowdiv, R, ldr, row0, c.kf, c.kh1,
                           vcol, vval, vnnz, c.vcap, flags);
    } else {
        const KrSlab sl = kr_slab(c.kf, c.kh1);
        hipLaunchKernelGGL(kreciprocal_generic_kernel, dim3((unsigned)(n < GEN_WG ? n : GEN_WG)), dim3(256), 0, s, ds,
                           rowdiv, R, ldr, row0, n, c.kf, c.kh1, sl, krslab, vcol, vval, vnnz, c.vcap, flags);
    }
    RM_LAUNCHED();
    return OK;
}

// Jaccard over unsorted inverted lists: every chunk scans whole lists and filters rows.
__global__ __launch_bounds__(256) void jaccard_scan_kernel(const float* __restrict__ OD, int64_t ld,
                                                           const float* __restrict__ rowdiv, int64_t Q, int64_t N,
                                                           Rows Vq, const int64_t* __restrict__ off,
                                                           const int32_t* __restrict__ irow,
                                                           const uint16_t* __restrict__ ival, uint16_t lam16,
                                                           float lam_f, float* __restrict__ out, int64_t ldo) {
    __shared__ uint16_t tmin[JCH];
    const int64_t i = blockIdx.y;
    const int64_t base = Q + (int64_t)blockIdx.x * JCH;
    const int64_t end = base + JCH < N ? base + JCH : N;
    const int span = (int)(end - base);
    for (int t = threadIdx.x; t < span; t += blockDim.x) tmin[t] = 0;
    __syncthreads();
    const int nz = Vq.len(i);
    const int64_t qb = Vq.beg(i);
    for (int e = 0; e < nz; e++) {
        const int32_t c = Vq.col[qb + e];
        const float vi = h2f_bits(Vq.val[qb + e]);
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

// od rows: OD (N x N, row i = distances from item i, scaled by 1/rowdiv[i] on the fly).
static int rerank_core(const float* OD, int64_t N, int64_t Q, int k1, int k2, uint16_t lam16, float lam_f,
                       float* out, int64_t ldo, char* ws, const RrPlan& P, int32_t* flags, hipStream_t s) {
    const RrCaps& c = P.caps;
    float* rmax = (float*)(ws + P.rowmax);
    int32_t* R = (int32_t*)(ws + P.rank);
    hipLaunchKernelGGL(rowmax_kernel, dim3(ceil_div(N, 4)), dim3(256), 0, s, OD, N, N, N, rmax);
    RM_LAUNCHED();
    int rc;
    if ((rc = topk_launch(OD, N, N, N, rmax, c.K, R, nullptr, c.K, s))) return rc;
    int32_t* vcol = (int32_t*)(ws + P.vcol);
    uint16_t* vval = (uint16_t*)(ws + P.vval);
    int32_t* vnnz = (int32_t*)(ws + P.vnnz);
    const DistSrc ds{OD, N, 0, nullptr, 0, 0, nullptr};
    if ((rc = v_rows_launch(ds, rmax, R, c.K, 0, N, c, ws + P.krslab, vcol, vval, vnnz, flags, s))) return rc;
    Rows Vq{nullptr, vnnz, c.vcap, vcol, vval};
    if (k2 != 1) {
        int32_t* qcol = (int32_t*)(ws + P.qcol);
        uint16_t* qval = (uint16_t*)(ws + P.qval);
        int32_t* qnnz = (int32_t*)(ws + P.qnnz);
        int32_t* dlist = (int32_t*)(ws + P.dlist);
        int32_t* dcount = (int32_t*)(ws + P.dcount);
        const Rows V{nullptr, vnnz, c.vcap, vcol, vval};
        if (c.k2e <= QE_FAST_K2) {
            RM_CHECK_HIP(hipMemsetAsync(dcount, 0, 4, s));
            hipLaunchKernelGGL(qe_kernel, dim3((unsigned)N), dim3(256), 0, s, R, (int64_t)c.K, c.k2e, (int64_t)0, V, qcol,
                               qval, qnnz, c.qcap, dlist, dcount);
            RM_LAUNCHED();
        }
        // the rows qe_kernel deferred (or every row): their count is read on the device
        hipLaunchKernelGGL(qe_generic_kernel, dim3(GEN_WG), dim3(256), 0, s, R, (int64_t)c.K, c.k2e, (int64_t)0, V,
                           c.k2e <= QE_FAST_K2 ? (const int32_t*)dlist : nullptr,
                           c.k2e <= QE_FAST_K2 ? (const int32_t*)dcount : nullptr, N, 2, qcol,
                           qval, qnnz, c.qcap, (const int64_t*)nullptr, P.qe, ws + P.qeslab, c.tcap, flags);
        RM_LAUNCHED();
        Vq = Rows{nullptr, qnnz, c.qcap, qcol, qval};
    }
    int32_t* cnt = (int32_t*)(ws + P.cnt);
    int64_t* off = (int64_t*)(ws + P.off);
    int32_t* cur = (int32_t*)(ws + P.cur);
    RM_CHECK_HIP(hipMemsetAsync(cnt, 0, N * 4, s));
    RM_CHECK_HIP(hipMemsetAsync(cur, 0, N * 4, s));
    hipLaunchKernelGGL(csc_count_kernel, dim3((unsigned)N), dim3(256), 0, s, Vq, N, cnt);
    RM_LAUNCHED();
    hipLaunchKernelGGL(scan_kernel, dim3(1), dim3(1024), 0, s, cnt, N, off);
    RM_LAUNCHED();
    hipLaunchKernelGGL(csc_fill_kernel, dim3((unsigned)N), dim3(256), 0, s, Vq, N, off, cur,
                       (int32_t*)(ws + P.irow), (uint16_t*)(ws + P.ival));
    RM_LAUNCHED();
    const int64_t G = N - Q;
    if (Q > 0 && G > 0) {
        dim3 grid(ceil_div(G, JCH), (unsigned)Q);
        hipLaunchKernelGGL(jaccard_scan_kernel, grid, dim3(256), 0, s, OD, N, rmax, Q, N, Vq, off,
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
    if (Q < 0 || G < 0 || N <= 0 || k1 < 1 || k2 < 1) return -1;
    return rr_plan(N, k1, k2, !from_dist, from_dist && need_transpose).total;
}

REIDMI_API int reidmi_rerank(const float* feat, int64_t Q, int64_t G, int64_t D, int64_t ldf, int k1, int k2,
                             uint16_t one_minus_lambda_h, float lambda_f, float* final_dist, int64_t ldo, void* ws_,
                             int64_t ws_bytes, int32_t* flags, void* stream) {
    const int64_t N = Q + G;
    RM_REQUIRE(Q >= 0 && G >= 0 && N > 0 && D > 0 && ldf >= D && ldo >= G && flags && k1 >= 1 && k2 >= 1,
               "rerank: bad arguments");
    RM_REQUIRE(N < 0x7fffffff, "rerank: too many items");
    const RrPlan P = rr_plan(N, k1, k2, true, false);
    RM_REQUIRE(ws_bytes >= P.total, "rerank: workspace too small");
    hipStream_t s = (hipStream_t)stream;
    char* ws = (char*)ws_;
    float* Dm = (float*)(ws + P.dist);
    int rc;
    // R1: exact-fp32 distance over cat(q, g); symmetric bit-for-bit (computed as the upper
    // triangle + its mirror), so od rows = D rows
    if ((rc = distmat_self_launch(feat, N, ldf, D, Dm, N, Dm + N * N, s))) return rc;
    return rerank_core(Dm, N, Q, k1, k2, one_minus_lambda_h, lambda_f, final_dist, ldo, ws, P, flags, s);
}

REIDMI_API int reidmi_rerank_from_dist(const float* dist, const float* add, int64_t Q, int64_t G, int symmetric,
                                       int k1, int k2, uint16_t one_minus_lambda_h, float lambda_f, float* final_dist,
                                       int64_t ldo, void* ws_, int64_t ws_bytes, int32_t* flags, void* stream) {
    const int64_t N = Q + G;
    RM_REQUIRE(Q >= 0 && G >= 0 && N > 0 && ldo >= G && flags && k1 >= 1 && k2 >= 1,
               "rerank_from_dist: bad arguments");
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

// dlist[t] = t for t < n, *dcount = n (every row deferred)
__global__ void iota_kernel(int32_t* __restrict__ dlist, int64_t n, int32_t* __restrict__ dcount) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < n) dlist[t] = (int32_t)t;
    if (t == 0) *dcount = (int32_t)n;
}

// ------------------------------------------------- small row utilities (staged R2)
// Ordered compaction: idx[0 .. *count) = the positions p < n with flags[p] != 0, ascending
// (np.nonzero).  One 1024-thread workgroup: each pass ballots 1024 flags, the waves' counts
// are scanned in LDS.
__global__ __launch_bounds__(1024) void nonzero_kernel(const int32_t* __restrict__ flags, int64_t n,
                                                       int32_t* __restrict__ idx, int32_t* __restrict__ count) {
    __shared__ int wsum[16];
    __shared__ int s_base;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    if (threadIdx.x == 0) s_base = 0;
    __syncthreads();
    for (int64_t p0 = 0; p0 < n; p0 += 1024) {
        const int64_t p = p0 + threadIdx.x;
        const bool k = p < n && flags[p] != 0;
        const uint64_t m = __ballot(k);
        if (lane == 0) wsum[wv] = __popcll(m);
        __syncthreads();
        int before = s_base;
        for (int w = 0; w < wv; w++) before += wsum[w];
        if (k) idx[before + __popcll(m & ((1ull << lane) - 1ull))] = (int32_t)p;
        __syncthreads();
        if (threadIdx.x == 0) {
            int t = 0;
            for (int w = 0; w < 16; w++) t += wsum[w];
            s_base += t;
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) *count = s_base;
}

// out[r][:] = x[row0 + idx[r]][:] (fp32 rows of d floats, 16-byte loads when aligned)
__global__ void gather_rows_kernel(const float* __restrict__ x, int64_t ldx, int64_t d, int64_t row0,
                                   const int32_t* __restrict__ idx, float* __restrict__ out, int64_t ldo) {
    const int64_t r = blockIdx.x;
    const float* src = x + (row0 + idx[r]) * ldx;
    float* dst = out + r * ldo;
    for (int64_t c = threadIdx.x; c < d; c += blockDim.x) dst[c] = src[c];
}

// ------------------------------------------------------------ staged re-ranking
// The same R1-R7 as row-range stages over caller-allocated, exactly sized buffers, so the
// N x N distance is never materialised (row chunks of it are) and the rows can be sharded
// over ranks with all-gathers between stages (multimodal_reid_amd/reranking.py).
REIDMI_API int reidmi_rr_caps(int64_t N, int k1, int k2, int64_t* vcap, int64_t* qcap, int64_t* v_ws_bytes,
                              int64_t* qe_ws_bytes) {
    RM_REQUIRE(N > 0 && k1 >= 1 && k2 >= 1 && vcap && qcap, "rr_caps: bad arguments");
    const RrCaps c = rr_caps(N, k1, k2);
    *vcap = c.vcap;
    *qcap = QCAP;
    if (v_ws_bytes) *v_ws_bytes = c.kr_fast ? 0 : GEN_WG * kr_slab(c.kf, c.kh1).bytes;
    if (qe_ws_bytes) *qe_ws_bytes = GEN_WG * qe_slab(c.k2e, c.tcap).bytes;
    return OK;
}

REIDMI_API int reidmi_rr_rank_rows(const float* feat, int64_t N, int64_t D, int64_t ldf, const float* sqn, int64_t lo,
                                   int64_t hi, int K, int32_t* rank_out, float* rowmax_out, float* chunk,
                                   int64_t chunk_rows, void* stream) {
    RM_REQUIRE(N > 0 && D > 0 && ldf >= D && 0 <= lo && lo <= hi && hi <= N && chunk_rows > 0 && K >= 1 && K <= N,
               "rr_rank_rows: bad arguments");
    RM_REQUIRE(N < 0x7fffffff, "rr_rank_rows: too many items");
    hipStream_t s = (hipStream_t)stream;
    int rc;
    for (int64_t a = lo; a < hi; a += chunk_rows) {
        const int64_t nb = hi - a < chunk_rows ? hi - a : chunk_rows;
        if ((rc = distmat_pre_launch(feat + a * ldf, nb, ldf, feat, N, ldf, D, sqn + a, sqn, chunk, N, s))) return rc;
        hipLaunchKernelGGL(rowmax_kernel, dim3(ceil_div(nb, 4)), dim3(256), 0, s, chunk, nb, N, N, rowmax_out + (a - lo));
        RM_LAUNCHED();
        if ((rc = topk_launch(chunk, nb, N, N, rowmax_out + (a - lo), K, rank_out + (a - lo) * K, nullptr, K, s)))
            return rc;
    }
    return OK;
}

// fp16 copy of the features for reidmi_rr_rank_rows_f16: [Np][Dp] (Np a multiple of 256 >= N,
// Dp a multiple of 64 >= D), zero-padded; *range_ok (device int32, set to 1 by the caller) is
// cleared when some |x| > 2^15 or is not finite (the pre-filter must not be used then).
REIDMI_API int reidmi_rr_feat16(const float* feat, int64_t N, int64_t D, int64_t ldf, void* feat16, int64_t Np,
                                int64_t Dp, int32_t* range_ok, void* stream) {
    RM_REQUIRE(Np % 256 == 0 && Dp % 64 == 0, "rr_feat16: Np % 256 == 0 and Dp % 64 == 0");
    return feat16_launch(feat, N, D, ldf, feat16, Np, Dp, range_ok, (hipStream_t)stream);
}

// Largest norm and squared norm over the items (out2[0], out2[1], device) for
// reidmi_rr_rank_rows_f16; once per feature set.
REIDMI_API int reidmi_rr_norm_max(const float* sqn, const float* nrm, int64_t N, float* out2, void* stream) {
    return norm_max_launch(sqn, nrm, N, out2, (hipStream_t)stream);
}

// Sampled survivor form of the pre-filter (backend.hip rr_sample_kernel / rank_select_sv_kernel):
// the sample is every S-th item, ns = floor(N / S) rounded down to whole 256-column tiles; per
// row: the sample's bounds, then the survivor list (RR_SV_CAP pairs) instead of an N-wide row.
// The selection runs inside the GEMM's epilogue (gemm.hip rrsv_tile): survivors staged in LDS,
// row / column records by LDS-DMA, no global memory instruction per tile.  A first version
// appended straight to the rows' lists (an atomic round trip per row group and tile, its
// registers spilling the K-loop): 13.0 s at N = 1.01 M against 3.9 + 1.7 s for the dense form
// (profiles/r03/rerank_1m_in_epilogue.txt).  Staged in LDS: 3.7 s for all row passes; over
// the symmetric product's upper triangle (each pair tested for both its rows, one call):
// 1.98 s, the 1M re-rank 7.1 -> 4.3 s (profiles/r03/rerank_1m_triangle.txt).
constexpr int RR_SAMPLE_STRIDE = 16, RR_SV_CAP_ = 4096;

__global__ void rr_gather_norms_kernel(const float* __restrict__ sqn, const float* __restrict__ nrm, int64_t ns,
                                       int S, float* __restrict__ sqn_s, float* __restrict__ nrm_s) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < ns) {
        sqn_s[t] = sqn[t * S];
        nrm_s[t] = nrm[t * S];
    }
}

// the survivor epilogue's column records (gemm.hip rrsv_tile) of the rectangular form: (squared
// norm, norm, -, -) of item c, zero past N
__global__ void rr_colrec_kernel(const float* __restrict__ sqn, const float* __restrict__ nrm, int64_t N, int64_t Np,
                                 float4* __restrict__ out) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < Np) out[t] = t < N ? make_float4(sqn[t], nrm[t], 0.f, 0.f) : make_float4(0.f, 0.f, 0.f, 0.f);
}

// The survivor GEMM's tile lists (gemm.h rr_tiles: M-tile << 16 | N-tile), bands of RR_BAND
// M-tiles walked N-major (the 32 tiles an XCD runs at once share 8 A and 4 W panels).
// Rectangular: tm x tn tiles.  Triangle (A = W, the whole symmetric product): the tiles with
// M-tile <= N-tile; band b (rows r0 = b B .. r0 + r - 1) holds, for N-tile nt >= r0,
// min(r, nt - r0 + 1) tiles.
constexpr int RR_BAND = 8;
__global__ void rr_rect_tiles_kernel(int tm, int tn, int* __restrict__ out) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (int64_t)tm * tn) return;
    const int per = RR_BAND * tn, b = (int)(t / per), r = (int)(t - (int64_t)b * per);
    const int rows = tm - b * RR_BAND < RR_BAND ? tm - b * RR_BAND : RR_BAND;
    const int nt = r / rows, mt = b * RR_BAND + r - nt * rows;
    out[t] = mt << 16 | nt;
}

__host__ __device__ inline int64_t rr_tri_band_count(int T, int b) {
    const int64_t r0 = (int64_t)b * RR_BAND, r = T - r0 < RR_BAND ? T - r0 : RR_BAND;
    return r * (r + 1) / 2 + (T - r0 - r) * r;
}

static int64_t rr_tri_tiles(int T) {
    int64_t n = 0;
    for (int b = 0; b * RR_BAND < T; b++) n += rr_tri_band_count(T, b);
    return n;
}

__global__ void rr_tri_tiles_kernel(int T, int* __restrict__ out) {
    const int b = blockIdx.x;
    __shared__ int64_t s_off;
    if (threadIdx.x == 0) {
        int64_t o = 0;
        for (int c = 0; c < b; c++) o += rr_tri_band_count(T, c);
        s_off = o;
    }
    __syncthreads();
    const int r0 = b * RR_BAND, r = T - r0 < RR_BAND ? T - r0 : RR_BAND;
    for (int nt = r0 + threadIdx.x; nt < T; nt += blockDim.x) {
        const int64_t k = nt - r0;
        const int64_t pos = s_off + (k < r ? k * (k + 1) / 2 : (int64_t)r * (r + 1) / 2 + (k - r) * r);
        const int c = k + 1 < r ? (int)k + 1 : r;
        for (int q = 0; q < c; q++) out[pos + q] = (r0 + q) << 16 | nt;
    }
}

// bytes of chunk the sampled form needs.  Rectangular (row passes): the column records, the
// sample's norms and the pass's tile list once, then per row the sample bounds, the survivor
// list, its counter, bound width and row record (the records padded to whole 256-row tiles:
// the epilogue's DMA reads them by tile).  Triangle (all rows in one call): the records of all
// items, the sample's norms, the tile list, the counters and widths, and the survivor lists of
// all rows (the sample bounds of a pass of rows overlay the lists before they are written).
static int64_t rr_sv_ns(int64_t N, int S) { return S >= 2 ? N / S / 256 * 256 : 0; }
static int64_t rr_sv_row_bytes(int64_t ns) { return 4 * ns + 8 * (int64_t)RR_SV_CAP_ + 4 + 4 + 16; }
// rows per pass of the rectangular form in a chunk of chunk_rows x Np floats (0: not applicable)
static int64_t rr_sv_pass_rows(int64_t N, int64_t Np, int64_t chunk_rows, int K, int S) {
    const int64_t ns = rr_sv_ns(N, S);
    if (ns < 256 || ns < 4 * K) return 0;
    // (the tile list of a pass of up to 65536 rows: 256 x Np / 256 ints = 4 Np bytes)
    const int64_t avail = chunk_rows * Np * 4 - 16 * Np - 8 * ns - 4 * Np - 256 * 16 - 256;
    int64_t r = avail / rr_sv_row_bytes(ns);
    r = r < 65536 ? r : 65536;
    return r >= 256 ? r / 256 * 256 : r >= 64 ? r : 0;  // whole 256-row tiles per pass when possible
}
// survivor capacity per row of the triangle form (0: not applicable: a list below 1024 pairs)
static int64_t rr_tri_cap(int64_t N, int64_t Np, int64_t chunk_rows, int K, int S) {
    const int64_t ns = rr_sv_ns(N, S);
    if (ns < 256 || ns < 4 * K || Np / 256 > 65536) return 0;
    const int64_t avail = chunk_rows * Np * 4 - 16 * Np - 8 * ns - 4 * rr_tri_tiles((int)(Np / 256)) - 8 * N - 1024;
    int64_t cap = avail / (8 * N) / 64 * 64;
    cap = cap < RR_SV_CAP_ ? cap : RR_SV_CAP_;
    return cap >= 1024 && 8 * N * cap >= 4 * ns * 256 ? cap : 0;
}

// ---- pieces of the triangle form, shared by rank_rows_f16 (one call over all rows) and the
// staged entry points reidmi_rr_tri_* (the sharded R2: the tile list split over ranks, the
// survivor lists of other ranks' rows exchanged, reranking.HipStages)
// sample norms (every S-th item), the upper-triangle tile list, the zero records past N
static int tri_init(const float* sqn, const float* nrm, int64_t N, int64_t Np, int64_t ns, int S, float4* meta,
                    float* sqn_s, float* nrm_s, int* tiles, hipStream_t s) {
    const int T = (int)(Np / 256);
    hipLaunchKernelGGL(rr_gather_norms_kernel, dim3((unsigned)ceil_div(ns, 256)), dim3(256), 0, s, sqn, nrm, ns, S,
                       sqn_s, nrm_s);
    RM_LAUNCHED();
    hipLaunchKernelGGL(rr_tri_tiles_kernel, dim3((unsigned)ceil_div(T, RR_BAND)), dim3(256), 0, s, T, tiles);
    RM_LAUNCHED();
    if (Np > N) RM_CHECK_HIP(hipMemsetAsync(meta + N, 0, (Np - N) * sizeof(float4), s));
    return OK;
}

// the sample's bounds of rows [a, a + nb) (EPI_RRHI against every S-th item) -> their records,
// widths and counters (rr_sample_kernel)
static int tri_sample(const _Float16* x16, int64_t Dp, const float* sqn, const float* nrm, const float* nmax2,
                      int64_t D, int K, int S, const float* sqn_s, const float* nrm_s, int64_t ns, int64_t a,
                      int64_t nb, float* hs, float4* meta, float* wrow, int32_t* cnt, int cap, hipStream_t s) {
    EpiArgs es{};
    es.out = hs;
    es.ldc = ns;
    es.rr_sqn = sqn;
    es.rr_nrm = nrm;
    es.rr_csqn = sqn_s;
    es.rr_cnrm = nrm_s;
    es.rr_row0 = a;
    es.rr_n = ns;
    rank_select_consts((int)D, es.rr_c);
    // the sample: W rows = every S-th item (row stride S * Dp)
    int r = gemm_f16(EPI_RRHI, x16 + a * Dp, Dp, x16, (int64_t)S * Dp, nb, ns, Dp, es, s);
    return r ? r : rr_sample_launch(hs, ns, ns, sqn, nrm, nmax2, a, nb, K, (int)D, meta, wrow, cnt, cap, s);
}

// the survivor GEMM (EPI_RRSV) over tiles [0, ntiles) of a tile list; tri: the list is (part
// of) the symmetric product's upper triangle and each pair above the diagonal is tested for both
// its rows
static int tri_survivors(const _Float16* x16, int64_t Dp, int64_t Np, const float* sqn, const float* nrm, int64_t N,
                         int64_t D, int64_t a, int64_t M, const float4* rowmeta, const float4* colrec, const int* tiles,
                         int64_t ntiles, bool tri, int32_t* cnt, int2* list, int cap, hipStream_t s) {
    if (ntiles <= 0) return OK;
    EpiArgs ev{};
    ev.rr_sqn = sqn;
    ev.rr_nrm = nrm;
    ev.rr_row0 = a;
    ev.rr_n = N;
    rank_select_consts((int)D, ev.rr_c);
    ev.rr_rowmeta = rowmeta;
    ev.rr_colrec = colrec;
    ev.rr_tiles = tiles;
    ev.rr_ntiles = ntiles;
    ev.rr_tri = tri;
    ev.sv_cnt = cnt;
    ev.sv_list = list;
    ev.sv_cap = cap;
    GemmOpts persistent;
    persistent.tile = 2;  // the survivor epilogue's LDS buffers live in the 256 x 256 tile
    return gemm_f16(EPI_RRSV, x16 + a * Dp, Dp, x16, Dp, M, Np, Dp, ev, s, persistent);
}

// rows per sample pass of the triangle form when its hs scratch overlays the N x cap lists
static int64_t tri_sample_rows(int64_t N, int64_t cap, int64_t ns) {
    return std::min<int64_t>(65536, 8 * N * cap / (4 * ns) / 256 * 256);
}

static int rank_rows_f16(const float* feat, int64_t N, int64_t D, int64_t ldf, const float* sqn, const float* nrm,
                         const float* nmax2, const void* feat16, int64_t Np, int64_t Dp, int64_t lo, int64_t hi,
                         int K, int32_t* rank_out, float* rowmax_out, int32_t* need, float* chunk,
                         int64_t chunk_rows, int S, hipStream_t s) {
    RM_REQUIRE(N > 0 && D > 0 && ldf >= D && 0 <= lo && lo <= hi && hi <= N && chunk_rows > 0 && K >= 1 && K <= N &&
                   K <= 64 && Np >= N && Np % 256 == 0 && Dp >= D && Dp % 64 == 0 && sqn && nrm && nmax2,
               "rr_rank_rows_f16: bad arguments");
    RM_REQUIRE(N < 0x7fffffff, "rr_rank_rows_f16: too many items");
    const _Float16* x16 = (const _Float16*)feat16;
    int rc;
    // (the survivor epilogue needs K >= 2 K-steps of the persistent tile: Dp >= 128)
    const bool sampled = Dp >= 128 && rr_sv_pass_rows(N, Np, chunk_rows, K, S) > 0;
    const int64_t tcap = sampled && lo == 0 && hi == N ? rr_tri_cap(N, Np, chunk_rows, K, S) : 0;
    const int T = (int)(Np / 256);
    auto sample = [&](float* hs, const float* sqn_s, const float* nrm_s, int64_t ns, int64_t a, int64_t nb,
                      float4* meta, float* wrow, int32_t* cnt, int cap) -> int {
        return tri_sample(x16, Dp, sqn, nrm, nmax2, D, K, S, sqn_s, nrm_s, ns, a, nb, hs, meta, wrow, cnt, cap, s);
    };
    auto survivors = [&](int64_t a, int64_t M, const float4* rowmeta, const float4* colrec, const int* tiles,
                         int64_t ntiles, bool tri, int32_t* cnt, int2* list, int cap) -> int {
        return tri_survivors(x16, Dp, Np, sqn, nrm, N, D, a, M, rowmeta, colrec, tiles, ntiles, tri, cnt, list, cap, s);
    };
    if (tcap > 0) {
        // triangle: every pair once (tiles with M-tile <= N-tile), tested for both its rows
        const int64_t ns = rr_sv_ns(N, S), ntri = rr_tri_tiles(T);
        float4* meta = (float4*)chunk;  // [Np]: row records = column records
        float* sqn_s = (float*)(meta + Np);
        float* nrm_s = sqn_s + ns;
        int* tiles = (int*)(nrm_s + ns);
        int32_t* cnt = (int32_t*)(tiles + ntri);
        float* wrow = (float*)(cnt + N);
        int2* list = (int2*)(((uintptr_t)(wrow + N) + 15) & ~(uintptr_t)15);  // [N][tcap]
        if ((rc = tri_init(sqn, nrm, N, Np, ns, S, meta, sqn_s, nrm_s, tiles, s))) return rc;
        const int64_t sp = tri_sample_rows(N, tcap, ns);  // rows per sample pass
        for (int64_t a = 0; a < N; a += sp) {
            const int64_t nb = N - a < sp ? N - a : sp;
            if ((rc = sample((float*)list, sqn_s, nrm_s, ns, a, nb, meta + a, wrow + a, cnt + a, (int)tcap))) return rc;
        }
        if ((rc = survivors(0, N, meta, meta, tiles, ntri, true, cnt, list, (int)tcap))) return rc;
        return rank_select_sv_launch(cnt, list, (int)tcap, wrow, feat, ldf, (int)D, sqn, 0, N, K, rank_out, rowmax_out,
                                     need, s);
    }
    if (sampled) {
        const int64_t pass = rr_sv_pass_rows(N, Np, chunk_rows, K, S);
        const int64_t ns = rr_sv_ns(N, S);
        float4* colrec = (float4*)chunk;  // [Np]
        float* sqn_s = (float*)(colrec + Np);
        float* nrm_s = sqn_s + ns;
        int* tiles = (int*)(nrm_s + ns);  // [pass / 256 (rounded up) x T]
        char* pbase = (char*)(((uintptr_t)(tiles + ceil_div(pass, 256) * (int64_t)T) + 15) & ~(uintptr_t)15);
        hipLaunchKernelGGL(rr_gather_norms_kernel, dim3((unsigned)ceil_div(ns, 256)), dim3(256), 0, s, sqn, nrm, ns, S,
                           sqn_s, nrm_s);
        RM_LAUNCHED();
        hipLaunchKernelGGL(rr_colrec_kernel, dim3((unsigned)ceil_div(Np, 256)), dim3(256), 0, s, sqn, nrm, N, Np,
                           colrec);
        RM_LAUNCHED();
        int tm_listed = -1;
        for (int64_t a = lo; a < hi; a += pass) {
            const int64_t nb = hi - a < pass ? hi - a : pass;
            float* hs = (float*)pbase;                                          // [nb][ns]
            int2* list = (int2*)(hs + nb * ns);                                 // [nb][cap]
            int32_t* cnt = (int32_t*)(list + nb * RR_SV_CAP_);                  // [nb]
            float* wrow = (float*)(cnt + nb);                                   // [nb]
            float4* meta = (float4*)(((uintptr_t)(wrow + nb) + 15) & ~(uintptr_t)15);  // [nb, padded to 256]
            const int tm = (int)ceil_div(nb, 256);
            if (tm != tm_listed) {
                hipLaunchKernelGGL(rr_rect_tiles_kernel, dim3((unsigned)ceil_div((int64_t)tm * T, 256)), dim3(256), 0, s,
                                   tm, T, tiles);
                RM_LAUNCHED();
                tm_listed = tm;
            }
            if ((rc = sample(hs, sqn_s, nrm_s, ns, a, nb, meta, wrow, cnt, RR_SV_CAP_))) return rc;
            if ((rc = survivors(a, nb, meta, colrec, tiles, (int64_t)tm * T, false, cnt, list, RR_SV_CAP_))) return rc;
            if ((rc = rank_select_sv_launch(cnt, list, RR_SV_CAP_, wrow, feat, ldf, (int)D, sqn, a, nb, K,
                                            rank_out + (a - lo) * K, rowmax_out + (a - lo), need + (a - lo), s)))
                return rc;
        }
        return OK;
    }
    for (int64_t a = lo; a < hi; a += chunk_rows) {
        const int64_t nb = hi - a < chunk_rows ? hi - a : chunk_rows;
        EpiArgs ea{};
        ea.out = chunk;
        ea.ldc = Np;
        ea.rr_sqn = sqn;
        ea.rr_nrm = nrm;
        ea.rr_row0 = a;
        ea.rr_n = N;
        rank_select_consts((int)D, ea.rr_c);
        if ((rc = gemm_f16(EPI_RRHI, x16 + a * Dp, Dp, x16, Dp, nb, Np, Dp, ea, s))) return rc;
        if ((rc = rank_select_launch(chunk, Np, feat, ldf, (int)D, sqn, nrm, nmax2, a, nb, N, K,
                                     rank_out + (a - lo) * K, rowmax_out + (a - lo), need + (a - lo), s)))
            return rc;
    }
    return OK;
}

// reidmi_rr_rank_rows with an fp16 pre-filter: the fp16 MFMA product of the rows with the
// items bounds every exact distance, and only each row's candidates are recomputed with the
// exact chain.  Same rank_out / rowmax_out bits as reidmi_rr_rank_rows for the rows with
// need[r] = 0; rows with need[r] = 1 (concentrated or non-finite distances) are left for the
// exact rows.  nrm = sqrt(sqn) [N]; nmax2 = reidmi_rr_norm_max of sqn, nrm.  chunk: chunk_rows x
// Np fp32 of scratch.  Default: sample stride RR_SAMPLE_STRIDE (16), the selection inside the
// GEMM's epilogue (backend.hip, "R2 pre-filter with the selection in the GEMM"; the triangle
// form when one call covers all rows); below that size, or with reidmi_rr_rank_rows_f16_ex's
// stride 0 / 1, the GEMM writes the rows' bounds (chunk_rows x Np) and rank_select1 streams them.
// Same bits either way.
REIDMI_API int reidmi_rr_rank_rows_f16(const float* feat, int64_t N, int64_t D, int64_t ldf, const float* sqn,
                                       const float* nrm, const float* nmax2, const void* feat16, int64_t Np,
                                       int64_t Dp, int64_t lo, int64_t hi, int K, int32_t* rank_out,
                                       float* rowmax_out, int32_t* need, float* chunk, int64_t chunk_rows,
                                       void* stream) {
    return rank_rows_f16(feat, N, D, ldf, sqn, nrm, nmax2, feat16, Np, Dp, lo, hi, K, rank_out, rowmax_out, need,
                         chunk, chunk_rows, RR_SAMPLE_STRIDE, (hipStream_t)stream);
}

// The same with the sample stride chosen (tests: 0 = the dense form at any N).
REIDMI_API int reidmi_rr_rank_rows_f16_ex(const float* feat, int64_t N, int64_t D, int64_t ldf, const float* sqn,
                                          const float* nrm, const float* nmax2, const void* feat16, int64_t Np,
                                          int64_t Dp, int64_t lo, int64_t hi, int K, int32_t* rank_out,
                                          float* rowmax_out, int32_t* need, float* chunk, int64_t chunk_rows,
                                          int sample_stride, void* stream) {
    RM_REQUIRE(sample_stride >= 0, "rr_rank_rows_f16_ex: sample_stride >= 0");
    return rank_rows_f16(feat, N, D, ldf, sqn, nrm, nmax2, feat16, Np, Dp, lo, hi, K, rank_out, rowmax_out, need,
                         chunk, chunk_rows, sample_stride, (hipStream_t)stream);
}

// Rows one pass of reidmi_rr_rank_rows_f16(_ex) takes with a chunk of chunk_rows x Np floats:
// the sampled form's pass (> chunk_rows for large N), or chunk_rows for the dense form.
// sample_stride < 0: the stride reidmi_rr_rank_rows_f16 uses.
REIDMI_API int64_t reidmi_rr_rank_rows_f16_pass_rows(int64_t N, int64_t Np, int64_t chunk_rows, int K,
                                                     int sample_stride) {
    if (N <= 0 || Np < N || chunk_rows <= 0 || K < 1) return -1;
    const int S = sample_stride < 0 ? RR_SAMPLE_STRIDE : sample_stride;
    if (rr_tri_cap(N, Np, chunk_rows, K, S) > 0) return N;  // one call over all rows: the triangle form
    const int64_t p = rr_sv_pass_rows(N, Np, chunk_rows, K, S);
    return p > 0 ? p : chunk_rows;
}

// ---- The triangle form of R2 in stages (reranking.HipStages' sharded R2): every
// rank samples its own rows (records all-gathered), runs a contiguous share of the upper-triangle
// tile list over ALL rows (each pair tested for both its rows), sends the partial survivor lists
// of other ranks' rows to their owners (reidmi_rr_sv_pack -> all-to-all -> reidmi_rr_sv_merge)
// and selects its own rows: the union of the lists is the one-call triangle form's, and the
// selection sorts each list by (hi, index), so the rows come out with the same bits for any
// number of ranks, at the one-GPU triangle's total MFMA work.
namespace reidmi {
__global__ void rr_sv_pack_kernel(const int32_t* __restrict__ cnt, const int2* __restrict__ list, int cap,
                                  int64_t rows, const int64_t* __restrict__ off, int2* __restrict__ out) {
    const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= rows) return;
    const int n = cnt[r] < cap ? cnt[r] : cap;
    const int2* src = list + r * cap;
    int2* dst = out + off[r];
    for (int p = threadIdx.x & 63; p < n; p += 64) dst[p] = src[p];
}

__global__ void rr_sv_merge_kernel(int32_t* __restrict__ cnt, int2* __restrict__ list, int cap, int64_t rows,
                                   const int32_t* __restrict__ add_cnt, const int64_t* __restrict__ add_off,
                                   const int2* __restrict__ add) {
    const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= rows) return;
    const int base = cnt[r], na = add_cnt[r];
    const int m = na < cap ? na : cap;  // entries the sender holds
    int2* dst = list + r * cap;
    const int2* src = add + add_off[r];
    for (int p = threadIdx.x & 63; p < m; p += 64)
        if ((int64_t)base + p < cap) dst[base + p] = src[p];
    __builtin_amdgcn_wave_barrier();
    if ((threadIdx.x & 63) == 0) {
        const int64_t t = (int64_t)base + na;
        cnt[r] = t < 0x3fffffff ? (int32_t)t : 0x3fffffff;  // > cap: the row overflows (need)
    }
}
}  // namespace reidmi

// Triangle form's sizes for a chunk of chunk_rows x Np floats (the same as the one-call form
// picks, reidmi_rr_rank_rows_f16): *ntiles = tiles of the upper triangle, *cap = survivor slots
// per row (0: the triangle form does not apply), *ns = sample items, *sample_rows = rows per
// sample pass when its scratch (sample_rows x ns fp32) overlays the N x cap lists.
REIDMI_API int reidmi_rr_tri_plan(int64_t N, int64_t Np, int64_t chunk_rows, int K, int64_t* ntiles, int64_t* cap,
                                  int64_t* ns, int64_t* sample_rows) {
    RM_REQUIRE(N > 0 && Np >= N && Np % 256 == 0 && chunk_rows > 0 && K >= 1 && ntiles && cap && ns && sample_rows,
               "rr_tri_plan: bad arguments");
    const int S = RR_SAMPLE_STRIDE;
    *cap = K <= 64 ? rr_tri_cap(N, Np, chunk_rows, K, S) : 0;
    *ns = rr_sv_ns(N, S);
    *ntiles = Np / 256 <= 65536 ? rr_tri_tiles((int)(Np / 256)) : 0;
    *sample_rows = *cap > 0 ? tri_sample_rows(N, *cap, *ns) : 0;
    return OK;
}

// meta [Np] float4 (row / column records; the tail past N zeroed here), sqn_s / nrm_s [ns],
// tiles [ntiles] int32 (the upper-triangle tile list, band order)
REIDMI_API int reidmi_rr_tri_init(const float* sqn, const float* nrm, int64_t N, int64_t Np, int64_t ns, void* meta,
                                  float* sqn_s, float* nrm_s, int32_t* tiles, void* stream) {
    RM_REQUIRE(sqn && nrm && meta && sqn_s && nrm_s && tiles && N > 0 && Np >= N && Np % 256 == 0 && ns >= 256 &&
                   ns * RR_SAMPLE_STRIDE <= N,
               "rr_tri_init: bad arguments");
    return tri_init(sqn, nrm, N, Np, ns, RR_SAMPLE_STRIDE, (float4*)meta, sqn_s, nrm_s, tiles, (hipStream_t)stream);
}

// Records, widths and counters of rows [a, b) (meta / wrow / cnt indexed by item): the sample's
// bounds in passes of hs_rows rows through hs (hs_rows x ns fp32; may overlay the lists).
REIDMI_API int reidmi_rr_tri_sample(const void* feat16, int64_t Np, int64_t Dp, const float* sqn, const float* nrm,
                                    const float* nmax2, int64_t N, int64_t D, int K, const float* sqn_s,
                                    const float* nrm_s, int64_t ns, int64_t a, int64_t b, float* hs, int64_t hs_rows,
                                    void* meta, float* wrow, int32_t* cnt, int cap, void* stream) {
    RM_REQUIRE(feat16 && sqn && nrm && nmax2 && sqn_s && nrm_s && hs && meta && wrow && cnt && 0 <= a && a <= b &&
                   b <= N && Np >= N && Dp >= D && Dp % 64 == 0 && K >= 1 && K <= 64 && hs_rows > 0 && ns >= K &&
                   cap >= 1 && cap <= RR_SV_CAP_,
               "rr_tri_sample: bad arguments");
    hipStream_t s = (hipStream_t)stream;
    int rc;
    for (int64_t x = a; x < b; x += hs_rows) {
        const int64_t nb = b - x < hs_rows ? b - x : hs_rows;
        if ((rc = tri_sample((const _Float16*)feat16, Dp, sqn, nrm, nmax2, D, K, RR_SAMPLE_STRIDE, sqn_s, nrm_s, ns, x, nb,
                             hs, (float4*)meta + x, wrow + x, cnt + x, cap, s)))
            return rc;
    }
    return OK;
}

// The survivor GEMM over tiles [t0, t1) of the triangle list, all N rows: appends to cnt [N] /
// list [N][cap] (cnt of rows not sampled on this rank must start at 0).
REIDMI_API int reidmi_rr_tri_survivors(const void* feat16, int64_t Np, int64_t Dp, const float* sqn, const float* nrm,
                                       int64_t N, int64_t D, const void* meta, const int32_t* tiles, int64_t t0,
                                       int64_t t1, int32_t* cnt, void* list, int cap, void* stream) {
    RM_REQUIRE(feat16 && sqn && nrm && meta && tiles && cnt && list && 0 <= t0 && t0 <= t1 && Np >= N && Np % 256 == 0 &&
                   Dp >= 128 && Dp % 64 == 0 && cap >= 1 && cap <= RR_SV_CAP_,
               "rr_tri_survivors: bad arguments");
    const float4* m = (const float4*)meta;
    return tri_survivors((const _Float16*)feat16, Dp, Np, sqn, nrm, N, D, 0, N, m, m, tiles + t0, t1 - t0, true, cnt,
                         (int2*)list, cap, (hipStream_t)stream);
}

// The selection of rows row0 .. row0 + rows from their lists (cnt / list / wrow indexed from
// row0): rank_out [rows][K], rowmax_out, need (rank_select_sv_kernel).
REIDMI_API int reidmi_rr_sv_select(const int32_t* cnt, const void* list, int cap, const float* wrow, const float* feat,
                                   int64_t ldf, int64_t D, const float* sqn, int64_t row0, int64_t rows, int K,
                                   int32_t* rank_out, float* rowmax_out, int32_t* need, void* stream) {
    RM_REQUIRE(cnt && list && wrow && feat && sqn && rank_out && rowmax_out && need && rows >= 0 && row0 >= 0,
               "rr_sv_select: bad arguments");
    return rank_select_sv_launch(cnt, (const int2*)list, cap, wrow, feat, ldf, (int)D, sqn, row0, rows, K, rank_out,
                                 rowmax_out, need, (hipStream_t)stream);
}

// The survivor lists of `rows` rows packed contiguously: out[off[r] + p] = list[r][p] for
// p < min(cnt[r], cap) (off = exclusive scan of those lengths).
REIDMI_API int reidmi_rr_sv_pack(const int32_t* cnt, const void* list, int cap, int64_t rows, const int64_t* off,
                                 void* out, void* stream) {
    RM_REQUIRE(cnt && list && off && rows >= 0 && cap >= 1 && (out || rows == 0), "rr_sv_pack: bad arguments");
    if (rows == 0) return OK;
    hipLaunchKernelGGL(rr_sv_pack_kernel, dim3((unsigned)ceil_div(rows, 4)), dim3(256), 0, (hipStream_t)stream, cnt,
                       (const int2*)list, cap, rows, off, (int2*)out);
    RM_LAUNCHED();
    return OK;
}

// Appends another rank's partial lists of the same rows: list[r][cnt[r] + p] = add[add_off[r] + p]
// while it fits cap; cnt[r] += add_cnt[r] (a total past cap marks the row's overflow, as the
// one-call form's counter does).
REIDMI_API int reidmi_rr_sv_merge(int32_t* cnt, void* list, int cap, int64_t rows, const int32_t* add_cnt,
                                  const int64_t* add_off, const void* add, void* stream) {
    RM_REQUIRE(cnt && list && add_cnt && add_off && rows >= 0 && cap >= 1, "rr_sv_merge: bad arguments");
    if (rows == 0) return OK;
    hipLaunchKernelGGL(rr_sv_merge_kernel, dim3((unsigned)ceil_div(rows, 4)), dim3(256), 0, (hipStream_t)stream, cnt,
                       (int2*)list, cap, rows, add_cnt, add_off, (const int2*)add);
    RM_LAUNCHED();
    return OK;
}

REIDMI_API int reidmi_rr_v_rows(const float* feat, int64_t N, int64_t D, int64_t ldf, const float* sqn,
                                const float* rowmax, const int32_t* rank, int K, int64_t lo, int64_t hi, int k1,
                                int32_t* vcol, uint16_t* vval, int32_t* vnnz, void* ws, int64_t ws_bytes,
                                int32_t* flags, void* stream) {
    RM_REQUIRE(N > 0 && D > 0 && ldf >= D && 0 <= lo && lo <= hi && hi <= N && flags, "rr_v_rows: bad arguments");
    RM_REQUIRE(k1 >= 1 && K >= (k1 + 1 < N ? k1 + 1 : N), "rr_v_rows: k1 >= 1, K >= min(k1 + 1, N)");
    const RrCaps c = rr_caps(N, k1, 1);
    RM_REQUIRE(c.kr_fast || (ws && ws_bytes >= GEN_WG * kr_slab(c.kf, c.kh1).bytes),
               "rr_v_rows: workspace of reidmi_rr_caps' v_ws_bytes required");
    const DistSrc ds{nullptr, 0, 0, feat, ldf, (int)D, sqn};
    return v_rows_launch(ds, rowmax, rank, K, lo, hi - lo, c, (char*)ws, vcol, vval, vnnz, flags, (hipStream_t)stream);
}

REIDMI_API int reidmi_rr_row_offsets(const int32_t* nnz, int64_t rows, int64_t* off, void* stream) {
    RM_REQUIRE(rows >= 0 && off, "rr_row_offsets: bad arguments");
    hipLaunchKernelGGL(scan_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, nnz, rows, off);
    RM_LAUNCHED();
    return OK;
}

REIDMI_API int reidmi_rr_pack(const int32_t* ell_col, const uint16_t* ell_val, const int32_t* nnz, int64_t rows,
                              int64_t cap, const int64_t* off, int32_t* col, uint16_t* val, void* stream) {
    RM_REQUIRE(rows >= 0 && cap > 0, "rr_pack: bad arguments");
    if (rows == 0) return OK;
    hipLaunchKernelGGL(rows_pack_kernel, dim3((unsigned)rows), dim3(256), 0, (hipStream_t)stream,
                       Rows{nullptr, nnz, cap, ell_col, ell_val}, off, col, val);
    RM_LAUNCHED();
    return OK;
}

// R4 main pass: rows lo..hi of V_qe into the ELL (qcol, qval, qnnz) of width
// reidmi_rr_caps' qcap; rows it cannot assemble in LDS get qnnz = 0 and are listed in
// dlist[0 .. *dcount) (dcount: device int32, cleared by the call) for reidmi_rr_qe_deferred.
REIDMI_API int reidmi_rr_qe_rows(const int32_t* rank, int K, int k2, int64_t lo, int64_t hi, const int64_t* voff,
                                 const int32_t* vcol, const uint16_t* vval, int32_t* qcol, uint16_t* qval,
                                 int32_t* qnnz, int32_t* dlist, int32_t* dcount, void* stream) {
    RM_REQUIRE(0 <= lo && lo <= hi && voff && dlist && dcount, "rr_qe_rows: bad arguments");
    RM_REQUIRE(k2 >= 2 && k2 <= K, "rr_qe_rows: 2 <= k2 <= K (k2 = 1 means V_qe = V)");
    hipStream_t s = (hipStream_t)stream;
    const int64_t n = hi - lo;
    if (k2 <= QE_FAST_K2) {
        RM_CHECK_HIP(hipMemsetAsync(dcount, 0, 4, s));
        if (n == 0) return OK;
        hipLaunchKernelGGL(qe_kernel, dim3((unsigned)n), dim3(256), 0, s, rank, (int64_t)K, k2, lo,
                           Rows{voff, nullptr, 0, vcol, vval}, qcol, qval, qnnz, (int64_t)QCAP, dlist, dcount);
        RM_LAUNCHED();
        return OK;
    }
    // k2 beyond the LDS kernel: every row is deferred
    RM_CHECK_HIP(hipMemsetAsync(qnnz, 0, n * 4, s));
    hipLaunchKernelGGL(iota_kernel, dim3(ceil_div(n > 0 ? n : 1, 256)), dim3(256), 0, s, dlist, n, dcount);
    RM_LAUNCHED();
    return OK;
}

// R4 for the rows deferred by reidmi_rr_qe_rows (dlist[0 .. n_def), relative to lo), on the
// workspace slabs (reidmi_rr_caps' qe_ws_bytes for the same N, k1, k2): mode 0 writes their
// entry counts to qnnz[b]; mode 1 writes the rows to CSR at qoff[b] (qoff: offsets of rows lo..hi).
REIDMI_API int reidmi_rr_qe_deferred(const int32_t* rank, int K, int k1, int k2, int64_t lo, int64_t N,
                                     const int64_t* voff, const int32_t* vcol, const uint16_t* vval,
                                     const int32_t* dlist, int64_t n_def, int mode, const int64_t* qoff, int32_t* qcol,
                                     uint16_t* qval, int32_t* qnnz, void* ws, int64_t ws_bytes, int32_t* flags,
                                     void* stream) {
    RM_REQUIRE(lo >= 0 && N > 0 && k1 >= 1 && voff && n_def >= 0 && (mode == 0 || mode == 1) && flags,
               "rr_qe_deferred: bad arguments");
    RM_REQUIRE(k2 >= 2 && k2 <= K, "rr_qe_deferred: 2 <= k2 <= K");
    RM_REQUIRE(mode == 0 ? qnnz != nullptr : (qoff && qcol && qval), "rr_qe_deferred: outputs");
    if (n_def == 0) return OK;
    RM_REQUIRE(dlist && n_def < (1ll << 31), "rr_qe_deferred: dlist");
    const RrCaps c = rr_caps(N, k1, k2);
    const QeSlab sl = qe_slab(k2, c.tcap);
    RM_REQUIRE(ws && ws_bytes >= GEN_WG * sl.bytes, "rr_qe_deferred: workspace of reidmi_rr_caps' qe_ws_bytes required");
    hipLaunchKernelGGL(qe_generic_kernel, dim3((unsigned)(n_def < GEN_WG ? n_def : GEN_WG)), dim3(256), 0,
                       (hipStream_t)stream, rank, (int64_t)K, k2, lo, Rows{voff, nullptr, 0, vcol, vval}, dlist,
                       (const int32_t*)nullptr, n_def, mode, qcol, qval, qnnz, (int64_t)0, qoff, sl, (char*)ws, c.tcap,
                       flags);
    RM_LAUNCHED();
    return OK;
}

namespace reidmi {
struct CscPlan {
    int64_t cnt, cur, sk, sv, total;
};
static CscPlan csc_plan(int64_t N, int64_t nnz) {
    CscPlan p{};
    int64_t o = 0;
    p.cnt = o; o = al(o + N * 4);
    p.cur = o; o = al(o + N * 4);
    p.sk = o; o = al(o + 2 * nnz * 4);  // padded sort scratch of long lists
    p.sv = o; o = al(o + 2 * nnz * 2);
    p.total = o;
    return p;
}
}  // namespace reidmi

REIDMI_API int64_t reidmi_rr_csc_workspace_bytes(int64_t N, int64_t nnz) { return csc_plan(N, nnz).total; }

// R5 for the staged driver: count per column, exclusive scan, atomic fill, per-column sort
// by row — the CSC of V_qe with every list in ascending row order (reranking.py:80-82).
REIDMI_API int reidmi_rr_csc(int64_t N, const int64_t* qoff, const int32_t* qcol, const uint16_t* qval, int64_t nnz,
                             int64_t* coff, int32_t* irow, uint16_t* ival, void* ws_, int64_t ws_bytes, void* stream) {
    RM_REQUIRE(N > 0 && N < (1ll << 31) && nnz >= 0 && nnz < 0x7fffffff && qoff && coff, "rr_csc: bad arguments");
    const CscPlan P = csc_plan(N, nnz);
    RM_REQUIRE(ws_bytes >= P.total, "rr_csc: workspace too small");
    hipStream_t s = (hipStream_t)stream;
    char* ws = (char*)ws_;
    const Rows V{qoff, nullptr, 0, qcol, qval};
    int32_t* cnt = (int32_t*)(ws + P.cnt);
    int32_t* cur = (int32_t*)(ws + P.cur);
    RM_CHECK_HIP(hipMemsetAsync(cnt, 0, N * 4, s));
    RM_CHECK_HIP(hipMemsetAsync(cur, 0, N * 4, s));
    hipLaunchKernelGGL(csc_count_kernel, dim3((unsigned)N), dim3(256), 0, s, V, N, cnt);
    RM_LAUNCHED();
    hipLaunchKernelGGL(scan_kernel, dim3(1), dim3(1024), 0, s, cnt, N, coff);
    RM_LAUNCHED();
    if (nnz == 0) return OK;
    hipLaunchKernelGGL(csc_fill_kernel, dim3((unsigned)N), dim3(256), 0, s, V, N, (const int64_t*)coff, cur, irow,
                       ival);
    RM_LAUNCHED();
    hipLaunchKernelGGL(csc_sort_kernel, dim3((unsigned)N), dim3(256), 0, s, (const int64_t*)coff, irow, ival,
                       (int32_t*)(ws + P.sk), (uint16_t*)(ws + P.sv));
    RM_LAUNCHED();
    return OK;
}

// bytes of the per-column chunk bounds of reidmi_rr_jaccard_rows (int64 per column and chunk
// boundary)
static int64_t jaccard_bounds_bytes(int64_t N, int64_t G) {
    const int64_t nch = (G + JCH - 1) / JCH;
    return N * (nch + 1) * 8;
}

REIDMI_API int64_t reidmi_rr_jaccard_bounds_bytes(int64_t N, int64_t G) {
    return N > 0 && G > 0 ? jaccard_bounds_bytes(N, G) : -1;
}

REIDMI_API int reidmi_rr_jaccard_rows(const float* feat, int64_t N, int64_t D, int64_t ldf, const float* sqn,
                                      const float* rowmax, int64_t Q, int64_t qlo, int64_t qhi, const int64_t* qoff,
                                      const int32_t* qcol, const uint16_t* qval, const int64_t* coff,
                                      const int32_t* irow, const uint16_t* ival, uint16_t one_minus_lambda_h,
                                      float lambda_f, float* out, int64_t ldo, float* chunk, int64_t chunk_rows,
                                      void* bounds, int64_t bounds_bytes, void* stream) {
    const int64_t G = N - Q;
    RM_REQUIRE(N > 0 && D > 0 && ldf >= D && 0 <= qlo && qlo <= qhi && qhi <= Q && Q <= N && ldo >= G &&
                   chunk_rows > 0 && chunk_rows <= 65535,
               "rr_jaccard_rows: bad arguments");
    if (qhi == qlo || G == 0) return OK;
    hipStream_t s = (hipStream_t)stream;
    const Rows Vq{qoff, nullptr, 0, qcol, qval};
    const int nch = ceil_div(G, JCH);
    RM_REQUIRE(bounds && ((uintptr_t)bounds & 7) == 0 && bounds_bytes >= jaccard_bounds_bytes(N, G),
               "rr_jaccard_rows: bounds of reidmi_rr_jaccard_bounds_bytes(N, N-Q) bytes (8-byte aligned) required");
    int64_t* cbnd = (int64_t*)bounds;
    hipLaunchKernelGGL(jaccard_bounds_kernel, dim3(ceil_div(N * (nch + 1), 256)), dim3(256), 0, s, coff, irow, N, Q,
                       nch, cbnd);
    RM_LAUNCHED();
    int rc;
    for (int64_t a = qlo; a < qhi; a += chunk_rows) {
        const int64_t nb = qhi - a < chunk_rows ? qhi - a : chunk_rows;
        // original_dist[a:a+nb, Q:N] (chunk, ld G)
        if ((rc = distmat_pre_launch(feat + a * ldf, nb, ldf, feat + Q * ldf, G, ldf, D, sqn + a, sqn + Q, chunk, G, s)))
            return rc;
        dim3 grid(ceil_div(G, JCH), (unsigned)nb);
        hipLaunchKernelGGL(jaccard_kernel, grid, dim3(256), 0, s, (const float*)chunk, G, Q, rowmax, a, Q, N, Vq, coff,
                           irow, ival, (const int64_t*)cbnd, one_minus_lambda_h, lambda_f, out + (a - qlo) * ldo, ldo);
        RM_LAUNCHED();
    }
    return OK;
}

// Row maxima skipping NaN (fmaxf), the od divisors of reranking.py:46 for a block of
// distance rows (rowmax_kernel).
REIDMI_API int reidmi_rowmax_f32(const float* x, int64_t rows, int64_t cols, int64_t ldx, float* out, void* stream) {
    RM_REQUIRE(rows >= 0 && cols > 0 && ldx >= cols && out, "rowmax: bad arguments");
    if (rows == 0) return OK;
    hipLaunchKernelGGL(rowmax_kernel, dim3(ceil_div(rows, 4)), dim3(256), 0, (hipStream_t)stream, x, rows, cols, ldx,
                       out);
    RM_LAUNCHED();
    return OK;
}

REIDMI_API int reidmi_nonzero_i32(const int32_t* flags, int64_t n, int32_t* idx, int32_t* count, void* stream) {
    RM_REQUIRE(n >= 0 && n < 0x7fffffff && count && (n == 0 || (flags && idx)), "nonzero: bad arguments");
    hipLaunchKernelGGL(nonzero_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, flags, n, idx, count);
    RM_LAUNCHED();
    return OK;
}

REIDMI_API int reidmi_gather_rows_f32(const float* x, int64_t ldx, int64_t d, int64_t row0, const int32_t* idx,
                                      int64_t n, float* out, int64_t ldo, void* stream) {
    RM_REQUIRE(n >= 0 && d > 0 && ldx >= d && ldo >= d && (n == 0 || (x && idx && out)), "gather_rows: bad arguments");
    if (n == 0) return OK;
    RM_REQUIRE(n < (1ll << 31), "gather_rows: too many rows");
    hipLaunchKernelGGL(gather_rows_kernel, dim3((unsigned)n), dim3(256), 0, (hipStream_t)stream, x, ldx, d, row0, idx,
                       out, ldo);
    RM_LAUNCHED();
    return OK;
}
