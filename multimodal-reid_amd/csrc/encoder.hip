// encoder.hip — CLIP vision / text towers of the CLIP-ReID eval path (gfx950).
//
// Elementwise/normalisation kernels (LayerNorm, on-the-fly TTA im2col, CLS/prompt rows,
// token embedding, EOT gather) and the host-side orchestration of one forward:
//   vision: custom_clip_model.VisionTransformer.forward (custom_clip_model.py:77-100),
//           IVLP maple.VisionTransformer.forward (maple.py:754-785, blocks maple.py:617-644)
//   text:   CLIP.encode_text (maple.py:971-984) / TextEncoder.forward (text_encoder.py:14-24)
// Per block: LN1 stats -> QKV GEMM (fp16, LN folded, head-split epilogue) -> fused MHSA ->
//            out_proj GEMM (+residual) -> LN2 stats -> c_fc GEMM (fp16, LN folded, +QuickGELU)
//            -> c_proj GEMM (+residual).
// The residual stream x is fp16 in HBM (the reference's GPU dtype, utils.py:145-166; every
// residual add is computed in fp32 and rounded once).  ln_1 / ln_2 never materialise: the
// QKV and c_fc GEMMs read x itself (fp16 operands) against W diag(gamma) and apply
// rstd * acc - mean * rstd * colsum + (b + W beta) in their epilogues (gemm.h).  Every other
// GEMM / attention operand (patch columns, q / k / v, softmax probabilities, attention and
// QuickGELU outputs, ln_post / ln_final rows) is fp16 too; LayerNorm statistics fp32.
#include "gemm.h"

namespace reidmi {

int mhsa(const void* q, const void* k, const void* vt, void* o, int64_t nseq, int L, int H, bool causal,
         hipStream_t s);
int attn_lpad(int L);
#ifdef REIDMI_TOOLS
// The fused QKV + attention kernel is bit-identical to the two-kernel block but measured slower
// at the bench batch (B = 1024, L = 211: 1.20 ms vs 1.09-1.12 ms for QKV GEMM + mhsa,
// tools/qkv_attn_ab.py, profiles/r03), so vision blocks run the two kernels and the kernel is
// built into the tools library only.
bool qkv_attn_fits(int L, int W, bool causal);
int qkv_attn(const void* x, int64_t ldx, const void* wq, int64_t ldw, const float* bias, const float* colsum,
             const void* rowstat, int64_t nseq, int L, int H, int W, void* o, hipStream_t s);
#endif
int mhsa_cls(const void* q, const void* k, const void* vt, void* o, int64_t nseq, int L, int H, hipStream_t s);
int64_t cls_attn_nokv_ws_bytes(int64_t nseq, int W);
int cls_attn_nokv(const void* x, const void* rs, const void* q, const void* wqkv, const float* colsum,
                  const float* bias, int64_t nseq, int L, int H, int W, void* ws, void* o, hipStream_t s);

// ------------------------------------------------------------------- LayerNorm
// One wave per row; W = NV*256, each lane holds NV groups of 4 consecutive elements.
// Two-pass mean/var in fp32 registers, eps inside the sqrt (torch.nn.LayerNorm).
// TX = float (public entry point) or _Float16 (the encoders' residual stream).
template <typename TX>
__device__ __forceinline__ float4 load4(const TX* p) {
    if constexpr (sizeof(TX) == 4) {
        return *(const float4*)p;
    } else {
        const f16x4 h = *(const f16x4*)p;
        return make_float4((float)h[0], (float)h[1], (float)h[2], (float)h[3]);
    }
}

template <int NV, typename TX>
__global__ __launch_bounds__(256) void layernorm_kernel(const TX* x, int64_t rows, int64_t ldx,
                                                        const int32_t* __restrict__ row_idx,
                                                        const float* __restrict__ gamma,
                                                        const float* __restrict__ beta, float eps,
                                                        float* __restrict__ y32, int64_t ldy32,
                                                        _Float16* __restrict__ y16, int64_t ldy16,
                                                        _Float16* yh, int64_t ldyh, float2* __restrict__ st,
                                                        float2* __restrict__ sto) {
    const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= rows) return;
    const int lane = threadIdx.x & 63;
    const int64_t src = row_idx ? (int64_t)row_idx[r] : r;
    const TX* xr = x + src * ldx;
    float4 v[NV];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NV; i++) {
        v[i] = load4(xr + 4 * (lane + 64 * i));
        s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
    }
    constexpr float invW = 1.0f / (NV * 256);
    const float mean = wave_sum(s) * invW;
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < NV; i++) {
        const float a = v[i].x - mean, b = v[i].y - mean, c = v[i].z - mean, d = v[i].w - mean;
        ss += (a * a + b * b) + (c * c + d * d);
    }
    const float rstd = __builtin_amdgcn_rsqf(wave_sum(ss) * invW + eps);
    if (st) {  // statistics for a LayerNorm folded into the next GEMM (gemm.h EpiArgs)
        if (lane == 0) st[r] = make_float2(rstd, -mean * rstd);
        return;
    }
#pragma unroll
    for (int i = 0; i < NV; i++) {
        const int f = lane + 64 * i;
        const float4 g = ((const float4*)gamma)[f], b = ((const float4*)beta)[f];
        float4 o;
        o.x = (v[i].x - mean) * rstd * g.x + b.x;
        o.y = (v[i].y - mean) * rstd * g.y + b.y;
        o.z = (v[i].z - mean) * rstd * g.z + b.z;
        o.w = (v[i].w - mean) * rstd * g.w + b.w;
        if (y32) ((float4*)(y32 + r * ldy32))[f] = o;
        if (y16) {
            f16x4 h = {(_Float16)o.x, (_Float16)o.y, (_Float16)o.z, (_Float16)o.w};
            ((f16x4*)(y16 + r * ldy16))[f] = h;
        }
        if (yh) {  // may alias x (in-place ln_pre): the whole row is in registers already
            f16x4 h = {(_Float16)o.x, (_Float16)o.y, (_Float16)o.z, (_Float16)o.w};
            ((f16x4*)(yh + r * ldyh))[f] = h;
            if (sto) v[i] = make_float4((float)h[0], (float)h[1], (float)h[2], (float)h[3]);
        }
    }
    if (sto) {  // statistics of the fp16 row just written (the next LayerNorm's, folded into a GEMM):
        // the same lane layout and summation order as the st pass over yh, so bit-identical to it
        float s2 = 0.f;
#pragma unroll
        for (int i = 0; i < NV; i++) s2 += (v[i].x + v[i].y) + (v[i].z + v[i].w);
        const float mean2 = wave_sum(s2) * invW;
        float ss2 = 0.f;
#pragma unroll
        for (int i = 0; i < NV; i++) {
            const float a = v[i].x - mean2, b = v[i].y - mean2, c = v[i].z - mean2, d = v[i].w - mean2;
            ss2 += (a * a + b * b) + (c * c + d * d);
        }
        const float rstd2 = __builtin_amdgcn_rsqf(wave_sum(ss2) * invW + eps);
        if (lane == 0) sto[r] = make_float2(rstd2, -mean2 * rstd2);
    }
}

template <typename TX>
int layernorm(const TX* x, int64_t rows, int64_t ldx, const int32_t* row_idx, int64_t W, const float* g,
              const float* b, float eps, float* y32, int64_t ldy32, _Float16* y16, int64_t ldy16, hipStream_t s,
              _Float16* yh = nullptr, int64_t ldyh = 0, float2* st = nullptr, float2* sto = nullptr) {
    if (rows == 0) return OK;
    RM_REQUIRE(ldx % 4 == 0 && (!y32 || ldy32 % 4 == 0) && (!y16 || ldy16 % 4 == 0) && (!yh || ldyh % 4 == 0),
               "layernorm: strides");
    RM_REQUIRE(!sto || (yh && !st), "layernorm: output statistics need the fp16 output");
    dim3 grid(ceil_div(rows, 4));
    switch (W) {
        case 512:
            hipLaunchKernelGGL((layernorm_kernel<2, TX>), grid, dim3(256), 0, s, x, rows, ldx, row_idx, g, b, eps, y32,
                               ldy32, y16, ldy16, yh, ldyh, st, sto);
            break;
        case 768:
            hipLaunchKernelGGL((layernorm_kernel<3, TX>), grid, dim3(256), 0, s, x, rows, ldx, row_idx, g, b, eps, y32,
                               ldy32, y16, ldy16, yh, ldyh, st, sto);
            break;
        case 1024:
            hipLaunchKernelGGL((layernorm_kernel<4, TX>), grid, dim3(256), 0, s, x, rows, ldx, row_idx, g, b, eps, y32,
                               ldy32, y16, ldy16, yh, ldyh, st, sto);
            break;
        default:
            return fail(EINVAL_, "layernorm: width must be 512, 768 or 1024");
    }
    RM_LAUNCHED();
    return OK;
}

// LayerNorm statistics only: st[r] = (rstd, -mean * rstd) of x row r (row stride ldx), the
// per-row half of a LayerNorm folded into the following fp16 GEMM.
static int row_stats(const _Float16* x, int64_t rows, int64_t ldx, int64_t W, float2* st, hipStream_t s) {
    return layernorm(x, rows, ldx, nullptr, W, nullptr, nullptr, 1e-5f, nullptr, 0, nullptr, 0, s, nullptr, 0, st);
}

// Row statistics from the residual epilogue's 64-column partials pst[b * rows + r]
// (Chan et al.'s pairwise combination): mean = sum / W, M2 = sum_b M2_b + 64 (mean_b - mean)^2, rstd = rsq(M2 / W +
// eps) -> st[r] = (rstd, -mean * rstd), replacing a statistics pass over x.
template <int NB>
__global__ __launch_bounds__(256) void rowstat_combine_kernel(const float2* __restrict__ pst, int64_t rows, float invw,
                                                              float eps, float2* __restrict__ st) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= rows) return;
    float2 v[NB];
#pragma unroll
    for (int b = 0; b < NB; b++) v[b] = pst[b * rows + r];
    float sum = 0.f;
#pragma unroll
    for (int b = 0; b < NB; b++) sum += v[b].x;
    const float mean = sum * invw;
    float m2 = 0.f;
#pragma unroll
    for (int b = 0; b < NB; b++) {
        const float d = v[b].x * (1.0f / 64) - mean;
        m2 += __builtin_fmaf(64.0f * d, d, v[b].y);
    }
    const float rstd = __builtin_amdgcn_rsqf(m2 * invw + eps);
    st[r] = make_float2(rstd, -mean * rstd);
}

static int row_stats_from_partials(const float2* pst, int64_t rows, int W, float2* st, hipStream_t s) {
    if (rows == 0) return OK;
    const dim3 g((unsigned)ceil_div(rows, 256)), t(256);
    switch (W) {
        case 512: hipLaunchKernelGGL(rowstat_combine_kernel<8>, g, t, 0, s, pst, rows, 1.0f / W, 1e-5f, st); break;
        case 768: hipLaunchKernelGGL(rowstat_combine_kernel<12>, g, t, 0, s, pst, rows, 1.0f / W, 1e-5f, st); break;
        case 1024: hipLaunchKernelGGL(rowstat_combine_kernel<16>, g, t, 0, s, pst, rows, 1.0f / W, 1e-5f, st); break;
        default: return fail(EINVAL_, "row statistics: width must be 512, 768 or 1024");
    }
    RM_LAUNCHED();
    return OK;
}

// fp16 residual rows -> fp32 output rows (x11 of encode_image / encode_cls)
__global__ void rows_f16_to_f32_kernel(const _Float16* __restrict__ x, int64_t rows, int64_t ldx, int W,
                                       float* __restrict__ y) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= rows * (W / 4)) return;
    const int64_t r = e / (W / 4);
    const int c = (int)(e % (W / 4)) * 4;
    *(float4*)(y + r * W + c) = load4(x + r * ldx + c);
}

// ---------------------------------------------------------- patch embed im2col
// col[b*NP + p][k], k = c*P*P + ky*P + kx (conv1.weight flattening), zero for k >= 3P^2.
// Optional TTA (data_prepare.py:263-270 on a normalised crop): flip, Pad((10,5)) with
// value -1 (= 0 before Normalize(0.5,0.5)), crop at (top i, left j).
// One workgroup per (image, patch row py): the P source rows of all 3 channels that the
// row's gw patches read (shifted by the TTA offset; rows outside the image = -1) are staged
// in LDS as fp16 (the output precision: fp32 inputs round once, here instead of at the store;
// 12 KB per workgroup at 256 x 128, so 8 workgroups share a CU) by coalesced 16-byte loads,
// then the gw * kpad outputs are written as
// 16-byte chunks (consecutive threads -> consecutive chunks).  The stride-S overlap (each
// pixel in up to 2x2 patches) is served from LDS, so HBM sees each image once.
// PT: the patch size as a compile-time constant (16: ViT-B/16, 14: ViT-L/14; 0 = runtime).
template <typename TI, int PT>
__global__ __launch_bounds__(256) void im2col_kernel(const TI* __restrict__ img, int H, int Wd, int P_, int S,
                                                     int gh, int gw, int kpad, const int32_t* __restrict__ tta,
                                                     _Float16* __restrict__ col) {
    extern __shared__ _Float16 srow[];  // [3][P][Wd]
    const int P = PT > 0 ? PT : P_;
    const int b = blockIdx.x / gh, py = blockIdx.x - (blockIdx.x / gh) * gh;
    const bool aug = tta != nullptr;
    const int ti = aug ? tta[2 * b] : 0, tj = aug ? tta[2 * b + 1] : 0;
    const int y0 = py * S + (aug ? ti - 5 : 0);
    const TI* im = img + (int64_t)b * 3 * H * Wd;
    constexpr int V = 16 / sizeof(TI);  // elements per 16-byte load (Wd % V == 0, checked at launch)
    const int vpr = Wd / V;             // loads per source row
    // fast: P % 8 == 0 and S % 4 == 0, so a col chunk is 8 consecutive staged pixels of one row at
    // an 8-byte aligned offset; the TTA view is then staged flipped and shifted (srow[cr][x'] = the
    // pixel the crop shows at column x': image column Wd - 1 - (x' + tj - 10), or -1 outside), and
    // both views read the stage the same way
    const bool fast = PT % 8 == 0 && PT > 0 && S % 4 == 0;
    if (fast && aug) {
        for (int e = threadIdx.x; e < 3 * P * vpr; e += blockDim.x) {
            const int cr = e / vpr, xv = e - cr * vpr;
            const int c = cr / P, y = y0 + (cr - c * P);
            _Float16 v[V];
            if (y >= 0 && y < H) {
                const uint4 raw = *(const uint4*)(im + ((int64_t)c * H + y) * Wd + xv * V);
                if constexpr (sizeof(TI) == 2) {
                    const f16x8 h = __builtin_bit_cast(f16x8, raw);
#pragma unroll
                    for (int u = 0; u < V; u++) v[u] = h[u];
                } else {
                    const float4 f = __builtin_bit_cast(float4, raw);
                    v[0] = (_Float16)f.x;
                    v[1] = (_Float16)f.y;
                    v[2] = (_Float16)f.z;
                    v[3] = (_Float16)f.w;
                }
            } else {
#pragma unroll
                for (int u = 0; u < V; u++) v[u] = (_Float16)-1.0f;
            }
#pragma unroll
            for (int u = 0; u < V; u++) {
                const int xp = Wd - 1 - (xv * V + u) - tj + 10;  // the crop column showing image column xv*V+u
                if (xp >= 0 && xp < Wd) srow[cr * Wd + xp] = v[u];
            }
        }
        // crop columns whose source lies outside the image (the Pad): -1
        const int nl = tj < 10 ? 10 - tj : 0, nr = tj > 10 ? tj - 10 : 0;
        for (int e = threadIdx.x; e < 3 * P * (nl + nr); e += blockDim.x) {
            const int cr = e / (nl + nr), u = e - cr * (nl + nr);
            srow[cr * Wd + (u < nl ? u : Wd - nr + (u - nl))] = (_Float16)-1.0f;
        }
    } else {
    for (int e = threadIdx.x; e < 3 * P * vpr; e += blockDim.x) {
        const int cr = e / vpr, xv = e - cr * vpr;  // cr = c * P + ky
        const int c = cr / P, y = y0 + (cr - c * P);
        _Float16* d = srow + cr * Wd + xv * V;
        if (y >= 0 && y < H) {
            const uint4 raw = *(const uint4*)(im + ((int64_t)c * H + y) * Wd + xv * V);
            if constexpr (sizeof(TI) == 2) {
                *(uint4*)d = raw;
            } else {
                const float4 f = __builtin_bit_cast(float4, raw);
                d[0] = (_Float16)f.x;
                d[1] = (_Float16)f.y;
                d[2] = (_Float16)f.z;
                d[3] = (_Float16)f.w;
            }
        } else {
#pragma unroll
            for (int u = 0; u < V; u++) d[u] = (_Float16)-1.0f;
        }
    }
    }
    __syncthreads();
    // PT > 0: kpad is the packed (3 P^2 + 63) / 64 * 64 (checked at launch), a compile-time chunk count
    const int kch = PT > 0 ? (3 * PT * PT + 63) / 64 * 8 : kpad / 8, PP = P * P;
    _Float16* out = col + ((int64_t)b * gh * gw + (int64_t)py * gw) * kpad;
    if (fast) {
        // a chunk's 8 k share (c, ky) and read 8 consecutive staged pixels, 8-byte aligned (row
        // stride Wd % 8 == 0, px * S * 2 bytes with S % 4 == 0)
        for (int e = threadIdx.x; e < gw * kch; e += blockDim.x) {
            const int px = e / kch, kc = e - px * kch, k0 = kc * 8;
            uint4 v = make_uint4(0u, 0u, 0u, 0u);
            if (k0 < 3 * PP) {
                const int c = k0 / PP, rem = k0 - c * PP, ky = rem / P, kx0 = rem - ky * P;
                const _Float16* src = srow + (c * P + ky) * Wd + px * S + kx0;
                const uint2 lo = *(const uint2*)src, hi = *(const uint2*)(src + 4);
                v = make_uint4(lo.x, lo.y, hi.x, hi.y);
            }
            *(uint4*)(out + (int64_t)px * kpad + kc * 8) = v;
        }
        return;
    }
    for (int e = threadIdx.x; e < gw * kch; e += blockDim.x) {
        const int px = e / kch, kc = e - px * kch;
        f16x8 o;
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const int k = kc * 8 + u;
            float v = 0.f;
            if (k < 3 * PP) {
                const int c = k / PP, rem = k - c * PP, ky = rem / P, kx = rem - ky * P;
                int x = px * S + kx;
                bool inb = true;
                if (aug) {
                    x = x + tj - 10;
                    inb = x >= 0 && x < Wd;
                    x = Wd - 1 - x;
                }
                v = inb ? (float)srow[(c * P + ky) * Wd + x] : -1.0f;
            }
            o[u] = (_Float16)v;
        }
        *(f16x8*)(out + (int64_t)px * kpad + kc * 8) = o;
    }
}

// x[b*L+0] = class_emb + pos[0]; IVLP: x[b*L+1+NP+i] = half(vpt[i]) (maple.py:765-767).
__global__ void cls_rows_kernel(_Float16* __restrict__ x, int64_t B, int L, int W, const float* __restrict__ cls,
                                const float* __restrict__ pos, int NP, int n_ctx, const float* __restrict__ vpt) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int rows = 1 + n_ctx;
    if (e >= B * rows * W) return;
    const int n = (int)(e % W);
    const int64_t br = e / W;
    const int64_t b = br / rows;
    const int r = (int)(br % rows);
    if (r == 0) x[(b * L) * W + n] = (_Float16)(cls[n] + pos[n]);
    else x[(b * L + 1 + NP + (r - 1)) * W + n] = (_Float16)vpt[(r - 1) * W + n];
}

// IVLP per-block prompt: rows [row0, row0+n_ctx) of every sequence <- half(prompt)
// (vision row0 = L-n_ctx, maple.py:620-629; text row0 = 1, maple.py:630-640).
__global__ void prompt_rows_kernel(_Float16* __restrict__ x, int64_t nseq, int L, int W, int row0, int n_ctx,
                                   const float* __restrict__ prompt) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= nseq * n_ctx * W) return;
    const int n = (int)(e % W);
    const int64_t br = e / W;
    const int64_t b = br / n_ctx;
    const int r = (int)(br % n_ctx);
    x[(b * L + row0 + r) * W + n] = (_Float16)prompt[r * W + n];
}

// x[n*L+t] = (prompts ? prompts[n,t] : tok_emb[tokens[n,t]]) + pos[t]   (maple.py:972-974),
// t < L; tokens / prompts rows have Lt >= L positions (the first L are used).
__global__ void text_embed_kernel(_Float16* __restrict__ x, const int64_t* __restrict__ tokens,
                                  const float* __restrict__ prompts, const float* __restrict__ tok_emb,
                                  const float* __restrict__ pos, int64_t N, int L, int Lt, int W, int64_t vocab) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= N * L * (W / 4)) return;
    const int c4 = (int)(e % (W / 4));
    const int64_t nt = e / (W / 4);
    const int t = (int)(nt % L);
    const int64_t src = (nt / L) * Lt + t;
    float4 v;
    if (prompts) v = ((const float4*)(prompts + src * W))[c4];
    else {
        int64_t id = tokens[src];
        id = id < 0 ? 0 : (id >= vocab ? vocab - 1 : id);
        v = ((const float4*)(tok_emb + id * W))[c4];
    }
    const float4 p = ((const float4*)(pos + (int64_t)t * W))[c4];
    const f16x4 h = {(_Float16)(v.x + p.x), (_Float16)(v.y + p.y), (_Float16)(v.z + p.z), (_Float16)(v.w + p.w)};
    ((f16x4*)(x + nt * W))[c4] = h;
}

// row index of tokens[n].argmax() over all Lt positions (first maximum, torch semantics) in
// the [N*L] row space (clamped to L-1: the caller's ctx_used covers every EOT position)
__global__ void eot_rows_kernel(const int64_t* __restrict__ tokens, int64_t N, int L, int Lt,
                                int32_t* __restrict__ rows) {
    const int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= N) return;
    const int64_t* t = tokens + n * Lt;
    int best = 0;
    int64_t bv = t[0];
    for (int i = 1; i < Lt; i++)
        if (t[i] > bv) { bv = t[i]; best = i; }
    rows[n] = (int32_t)(n * L + (best < L ? best : L - 1));
}

// --------------------------------------------------------------- workspace plan
struct Plan {
    int64_t x, h, q, k, vt, o, u, rows, st, st_cls, pst, total;
};

static int64_t al(int64_t v) { return (v + 255) & ~(int64_t)255; }

static Plan plan(int64_t nseq, int L, int W, int lp, int64_t extra_rows) {
    Plan p{};
    const int64_t M = nseq * L;
    int64_t off = 0;
    p.x = off; off = al(off + M * W * 2);  // fp16 residual stream
    p.h = off; off = al(off + M * W * 2);
    p.q = off; off = al(off + M * W * 2);
    p.k = off; off = al(off + M * W * 2);
    p.vt = off; off = al(off + nseq * W * (int64_t)lp * 2);
    p.o = off; off = al(off + M * W * 2);
    p.u = off; off = al(off + M * 4 * W * 2);
    p.rows = off; off = al(off + extra_rows * 4);
    // LayerNorm statistics of every row / of the CLS rows (run_block_cls), padded to whole
    // 256-row GEMM tiles (the folded GEMM reads them per tile, gemm.h)
    p.st = off; off = al(off + (M + 256) * 8);
    p.st_cls = off; off = al(off + (nseq + 256) * 8);
    // LayerNorm partials [W/64][M] (sum, centred sum of squares) written by the residual
    // GEMM epilogues (gemm.h EpiArgs::pstat)
    p.pst = off; off = al(off + M * (W / 64) * 8);
    p.total = off;
    return p;
}

// Where a block's ln_1 statistics come from: a pass over x (row_stats), the partials the
// previous block's c_proj epilogue wrote (x_pst), or already at P.st (ln_pre wrote them).
enum XStats { XS_ROWS = 0, XS_PARTIALS = 1, XS_READY = 2 };

static int ln1_stats(XStats xs, char* ws, const Plan& P, int64_t M, int W, hipStream_t s) {
    float2* st = (float2*)(ws + P.st);
    if (xs == XS_READY) return OK;
    if (xs == XS_PARTIALS) return row_stats_from_partials((const float2*)(ws + P.pst), M, W, st, s);
    return row_stats((const _Float16*)(ws + P.x), M, W, W, st, s);
}

// One ResidualAttentionBlock on the fp16 residual stream x [nseq*L][W].  ln_1 / ln_2 are
// folded into the QKV / c_fc GEMMs (fp16 operands: x itself and W diag(gamma)); only the
// per-row statistics are computed here (row_stats), never the normalised activations.
// xs: where ln_1's statistics come from (XStats); XS_PARTIALS when the partials at P.pst
// describe x as it is now (written by the previous block's c_proj epilogue, not overwritten since).
static int run_block(const reidmi_block_weights& bw, char* ws, const Plan& P, int64_t nseq, int L, int W, int H,
                     bool causal, XStats xs, hipStream_t s) {
    const int64_t M = nseq * L;
    float2* pst = (float2*)(ws + P.pst);
    _Float16* x = (_Float16*)(ws + P.x);
    _Float16* o = (_Float16*)(ws + P.o);
    _Float16* u = (_Float16*)(ws + P.u);
    float2* st = (float2*)(ws + P.st);
    int rc;
    // ln_1 (custom_clip_model.py:27)
    if ((rc = ln1_stats(xs, ws, P, M, W, s))) return rc;
    {
        EpiArgs ea{};
        ea.bias = bw.qkv_b;
        ea.rowstat = st;
        ea.colsum = bw.qkv_s;
        ea.q = ws + P.q;
        ea.k = ws + P.k;
        ea.vt = ws + P.vt;
        ea.seq = L;
        ea.heads = H;
        ea.lpad = attn_lpad(L);
        if ((rc = gemm_f16(EPI_QKV, x, W, bw.qkv_w, W, M, 3 * W, W, ea, s))) return rc;
        if ((rc = mhsa(ws + P.q, ws + P.k, ws + P.vt, o, nseq, L, H, causal, s))) return rc;
    }
    EpiArgs er{};
    er.out = x;
    er.ldc = W;
    er.bias = bw.out_b;
    er.pstat = pst;
    er.ldp = M;
    if ((rc = gemm_f16(EPI_RESID_F16, o, W, bw.out_w, W, M, W, W, er, s))) return rc;
    if ((rc = row_stats_from_partials(pst, M, W, st, s))) return rc;  // ln_2 (custom_clip_model.py:28)
    EpiArgs eg{};
    eg.out = u;
    eg.ldc = 4 * W;
    eg.bias = bw.fc1_b;
    eg.rowstat = st;
    eg.colsum = bw.fc1_s;
    if ((rc = gemm_f16(EPI_GELU_H16, x, W, bw.fc1_w, W, M, 4 * W, W, eg, s))) return rc;
    EpiArgs e2{};
    e2.out = x;
    e2.ldc = W;
    e2.bias = bw.fc2_b;
    e2.pstat = pst;  // for the next block's ln_1
    e2.ldp = M;
    if ((rc = gemm_f16(EPI_RESID_F16, u, 4 * W, bw.fc2_w, 4 * W, M, W, 4 * W, e2, s))) return rc;
    return OK;
}

__global__ void gather_rowstat_kernel(const float2* __restrict__ st, int64_t nseq, int L, float2* __restrict__ sc) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b < nseq) sc[b] = st[b * L];
}

// The last block when only the CLS row of its output is consumed (inference path,
// zero_shot_learning.py:85-87 reads x12[:,0] / xproj[:,0]): Q, attention, out_proj, LN2 and
// the MLP for the CLS rows only.  The CLS query's attention reads the ln_1 input x of every
// token directly (cls_attn_nokv, attention.hip: scores and the value sum reassociated through
// the folded in_proj, so K and V are never formed for the 211 tokens — round 5; the K / V GEMM +
// single-query kernel path of rounds 1-4 runs with REIDMI_CLS_KV=1, the A/B and test baseline).
// Its LayerNorm statistics come from a pass over the CLS rows, where run_block combines the
// residual epilogues' partials (a different fp32 summation order): equal to the full block's
// row 0 up to that rounding and the fp16 roundings of K / V it skips (tests/test_gpu_encoder.py
// bounds the difference).
static int run_block_cls(const reidmi_block_weights& bw, char* ws, const Plan& P, int64_t nseq, int L, int W, int H,
                         XStats xs, hipStream_t s) {
    const int64_t M = nseq * L;
    _Float16* x = (_Float16*)(ws + P.x);
    _Float16* o = (_Float16*)(ws + P.o);
    _Float16* u = (_Float16*)(ws + P.u);
    float2* st = (float2*)(ws + P.st);
    float2* sc = (float2*)(ws + P.st_cls);
    const int64_t ldc = (int64_t)L * W;  // CLS row of each sequence
    int rc;
    if ((rc = ln1_stats(xs, ws, P, M, W, s))) return rc;
    // the CLS rows' ln_1 statistics are rows b*L of st (so Q, K and V of a CLS row use the
    // same statistics); gathered into the padded per-sequence buffer the Q GEMM reads
    hipLaunchKernelGGL(gather_rowstat_kernel, dim3(ceil_div(nseq, 256)), dim3(256), 0, s, st, nseq, L, sc);
    RM_LAUNCHED();
    // the reassociated path covers widths 768 / 1024 (64-wide heads), L <= 224 and scratch that
    // fits the K buffer of the other path (L * W * 2 bytes per image); anything else (and
    // REIDMI_CLS_KV=1, read per call: tests switch it in-process) takes the K / V path
    const char* kv_env = getenv("REIDMI_CLS_KV");
    const bool kv_path = (kv_env != nullptr && kv_env[0] == '1') || !(W == 768 || W == 1024) || H * 64 != W ||
                         L > 224 || cls_attn_nokv_ws_bytes(nseq, W) > nseq * L * W * 2;
    EpiArgs qa{};
    qa.bias = bw.qkv_b;
    qa.rowstat = sc;
    qa.colsum = bw.qkv_s;
    qa.q = ws + P.q;
    qa.seq = 1;  // one (CLS) row per sequence: q [nseq*H][1][64]
    qa.heads = H;
    qa.lpad = 1;
    if (!kv_path) {
        if ((rc = gemm_f16(EPI_QKV, x, ldc, bw.qkv_w, W, nseq, W, W, qa, s))) return rc;
        if ((rc = cls_attn_nokv(x, st, ws + P.q, bw.qkv_w, bw.qkv_s, bw.qkv_b, nseq, L, H, W, ws + P.k, o, s)))
            return rc;
    } else {  // K and V for every token, then the single-query kernel
        EpiArgs kv{};
        kv.bias = bw.qkv_b + W;
        kv.rowstat = st;
        kv.colsum = bw.qkv_s + W;
        kv.k = ws + P.k;
        kv.vt = ws + P.vt;
        kv.seq = L;
        kv.heads = H;
        kv.lpad = attn_lpad(L);
        kv.n_off = W;
        if ((rc = gemm_f16(EPI_QKV, x, W, (const _Float16*)bw.qkv_w + (int64_t)W * W, W, M, 2 * W, W, kv, s)))
            return rc;
        if ((rc = gemm_f16(EPI_QKV, x, ldc, bw.qkv_w, W, nseq, W, W, qa, s))) return rc;
        if ((rc = mhsa_cls(ws + P.q, ws + P.k, ws + P.vt, o, nseq, L, H, s))) return rc;
    }
    EpiArgs er{};
    er.out = x;
    er.ldc = ldc;
    er.bias = bw.out_b;
    if ((rc = gemm_f16(EPI_RESID_F16, o, W, bw.out_w, W, nseq, W, W, er, s))) return rc;
    if ((rc = row_stats(x, nseq, ldc, W, sc, s))) return rc;
    EpiArgs eg{};
    eg.out = u;
    eg.ldc = 4 * W;
    eg.bias = bw.fc1_b;
    eg.rowstat = sc;
    eg.colsum = bw.fc1_s;
    if ((rc = gemm_f16(EPI_GELU_H16, x, ldc, bw.fc1_w, W, nseq, 4 * W, W, eg, s))) return rc;
    EpiArgs e2{};
    e2.out = x;
    e2.ldc = ldc;
    e2.bias = bw.fc2_b;
    return gemm_f16(EPI_RESID_F16, u, 4 * W, bw.fc2_w, 4 * W, nseq, W, 4 * W, e2, s);
}

static int vit_check(const reidmi_vit_weights* w) {
    RM_REQUIRE(w && w->blocks, "vit: null weights");
    RM_REQUIRE(w->layers >= 12, "vit: the reference forward runs resblocks[:11] + resblocks[11]; needs >= 12 layers");
    RM_REQUIRE(w->width == w->heads * 64, "vit: head dim must be 64");
    RM_REQUIRE(w->kpad % 64 == 0 && w->kpad >= 3 * w->patch * w->patch, "vit: kpad");
    RM_REQUIRE(w->out_dim % 128 == 0 && w->width % 128 == 0, "vit: width/out_dim must be multiples of 128");
    return OK;
}

}  // namespace reidmi

using namespace reidmi;

REIDMI_API int reidmi_layernorm(const float* x, int64_t rows, int64_t ldx, const int32_t* row_idx, int64_t W,
                                const float* gamma, const float* beta, float eps, float* y32, int64_t ldy32, void* y16,
                                int64_t ldy16, void* stream) {
    return layernorm(x, rows, ldx, row_idx, W, gamma, beta, eps, y32, ldy32, (_Float16*)y16, ldy16,
                     (hipStream_t)stream);
}

REIDMI_API int64_t reidmi_vit_workspace_bytes(const reidmi_vit_weights* w, int64_t B, int full) {
    if (vit_check(w)) return -1;
    const int L = 1 + w->grid_h * w->grid_w + w->n_ctx;
    return plan(B, L, w->width, attn_lpad(L), 0).total;
}

REIDMI_API int reidmi_vit_forward(const reidmi_vit_weights* w, const void* images, int images_f16, int64_t B, int H,
                                  int Wimg, const int32_t* tta, int full, float* out_x12, float* out_proj,
                                  float* out_x11, void* ws_, int64_t ws_bytes, void* stream) {
    int rc;
    if ((rc = vit_check(w))) return rc;
    hipStream_t s = (hipStream_t)stream;
    const int W = w->width, NP = w->grid_h * w->grid_w, L = 1 + NP + w->n_ctx, E = w->out_dim;
    RM_REQUIRE((H - w->patch) / w->stride + 1 == w->grid_h && (Wimg - w->patch) / w->stride + 1 == w->grid_w,
               "vit: image size does not match the positional-embedding grid");
    RM_REQUIRE(attn_lpad(L) > 0, "vit: too many tokens (max 256)");
    const Plan P = plan(B, L, W, attn_lpad(L), 0);
    RM_REQUIRE(ws_bytes >= P.total, "vit: workspace too small");
    RM_REQUIRE(out_x12 && out_proj, "vit: outputs required");
    if (B == 0) return OK;
    char* ws = (char*)ws_;
    _Float16* x = (_Float16*)(ws + P.x);
    _Float16* h = (_Float16*)(ws + P.h);
    _Float16* col = (_Float16*)(ws + P.u);
    const int64_t M = B * L;
    // patch embed (+pos), CLS/VPT rows, ln_pre
    RM_REQUIRE(B * w->grid_h < (1ll << 31) && Wimg % 8 == 0, "vit: im2col needs B * grid_h < 2^31 and width % 8 == 0");
    {
        const dim3 g((unsigned)(B * w->grid_h)), t(256);
        const size_t lds = (size_t)3 * w->patch * Wimg * sizeof(_Float16);
        RM_REQUIRE(lds <= 64 * 1024, "vit: image too wide for the im2col row stage");
#define RM_IM2COL(TI, PT)                                                                                      \
    hipLaunchKernelGGL((im2col_kernel<TI, PT>), g, t, lds, s, (const TI*)images, H, Wimg, w->patch, w->stride, \
                       w->grid_h, w->grid_w, w->kpad, tta, col)
        // the compile-time patch sizes assume the packed kpad (pack.hip)
        const int pt = w->kpad == (3 * w->patch * w->patch + 63) / 64 * 64 ? w->patch : 0;
        if (images_f16) {
            if (pt == 16) RM_IM2COL(_Float16, 16);
            else if (pt == 14) RM_IM2COL(_Float16, 14);
            else RM_IM2COL(_Float16, 0);
        } else {
            if (pt == 16) RM_IM2COL(float, 16);
            else if (pt == 14) RM_IM2COL(float, 14);
            else RM_IM2COL(float, 0);
        }
#undef RM_IM2COL
    }
    RM_LAUNCHED();
    EpiArgs ep{};
    ep.out = x;
    ep.ldc = W;
    ep.pos = w->pos_emb;
    ep.npatch = NP;
    ep.seq = L;
    if ((rc = gemm_f16(EPI_PATCH, col, w->kpad, w->conv_w, w->kpad, B * NP, W, w->kpad, ep, s))) return rc;
    RM_REQUIRE(w->n_ctx == 0 || w->vpt != nullptr, "vit: n_ctx > 0 needs vpt");
    const int64_t ce = B * (1 + w->n_ctx) * W;
    hipLaunchKernelGGL(cls_rows_kernel, dim3(ceil_div(ce, 256)), dim3(256), 0, s, x, B, L, W, w->class_emb,
                       w->pos_emb, NP, w->n_ctx, w->vpt);
    RM_LAUNCHED();
    // in place; also writes the statistics of its output rows, block 0's ln_1 (XS_READY)
    if ((rc = layernorm(x, M, W, nullptr, W, w->ln_pre_w, w->ln_pre_b, 1e-5f, nullptr, 0, nullptr, 0, s, x, W, nullptr,
                        (float2*)(ws + P.st))))
        return rc;
    // resblocks[:11] then resblocks[11] (custom_clip_model.py:91-92)
    for (int i = 0; i < 12; i++) {
        const reidmi_block_weights& bw = w->blocks[i];
        if (i > 0 && bw.prompt && w->n_ctx > 0) {
            const int64_t pe = B * w->n_ctx * W;
            hipLaunchKernelGGL(prompt_rows_kernel, dim3(ceil_div(pe, 256)), dim3(256), 0, s, x, B, L, W,
                               L - w->n_ctx, w->n_ctx, bw.prompt);
            RM_LAUNCHED();
        }
        // x's partials are current unless this is block 0 (ln_pre wrote x and its statistics)
        // or prompt rows were just overwritten (IVLP)
        const XStats xs = i == 0 ? XS_READY : (bw.prompt && w->n_ctx > 0) ? XS_ROWS : XS_PARTIALS;
        if (i == 11 && !full) rc = run_block_cls(bw, ws, P, B, L, W, w->heads, xs, s);
        else rc = run_block(bw, ws, P, B, L, W, w->heads, false, xs, s);
        if (rc) return rc;
        if (i == 10 && out_x11) {  // resblocks[:11] output (fp16 stream -> fp32)
            const int64_t r11 = full ? M : B;
            hipLaunchKernelGGL(rows_f16_to_f32_kernel, dim3(ceil_div(r11 * (W / 4), 256)), dim3(256), 0, s, x, r11,
                               full ? (int64_t)W : (int64_t)L * W, W, out_x11);
            RM_LAUNCHED();
        }
    }
    // ln_post, then @ proj (custom_clip_model.py:96-98)
    const int64_t rows = full ? M : B;
    const int64_t ldx = full ? W : (int64_t)L * W;
    if ((rc = layernorm(x, rows, ldx, nullptr, W, w->ln_post_w, w->ln_post_b, 1e-5f, out_x12, W, h, W, s))) return rc;
    EpiArgs eo{};
    eo.out = out_proj;
    eo.ldc = E;
    if ((rc = gemm_f16(EPI_F32, h, W, w->proj_t, W, rows, E, W, eo, s))) return rc;
    return OK;
}

REIDMI_API int64_t reidmi_text_workspace_bytes(const reidmi_text_weights* w, int64_t N) {
    if (!w || attn_lpad(w->ctx) < 0) return -1;
    return plan(N, w->ctx, w->width, attn_lpad(w->ctx), N).total;
}

REIDMI_API int reidmi_text_forward(const reidmi_text_weights* w, const int64_t* tokens, const float* prompts,
                                   int64_t N, int ctx_used, float* out, void* ws_, int64_t ws_bytes, void* stream) {
    RM_REQUIRE(w && w->blocks && tokens && out, "text: null argument");
    RM_REQUIRE(w->width == w->heads * 64 && w->width % 256 == 0, "text: width");
    hipStream_t s = (hipStream_t)stream;
    const int W = w->width, Lt = w->ctx, E = w->out_dim;
    // Causal mask: row t of every block reads rows <= t only, so the rows past the last EOT
    // position never reach the output (x[n, argmax(tokens[n])], maple.py:981); ctx_used > 0
    // runs the tower on the first ctx_used positions (the caller guarantees every EOT and
    // every IVLP prompt row lies below it) - the same values for the rows it keeps.
    const int L = ctx_used > 0 ? ctx_used : Lt;
    RM_REQUIRE(L <= Lt && L > w->n_ctx, "text: ctx_used must be in (n_ctx, ctx]");
    RM_REQUIRE(attn_lpad(L) > 0, "text: context too long");
    const Plan P = plan(N, L, W, attn_lpad(L), N);
    RM_REQUIRE(ws_bytes >= P.total, "text: workspace too small");
    if (N == 0) return OK;
    char* ws = (char*)ws_;
    _Float16* x = (_Float16*)(ws + P.x);
    _Float16* h = (_Float16*)(ws + P.h);
    int32_t* rows = (int32_t*)(ws + P.rows);
    const int64_t te = N * L * (W / 4);
    hipLaunchKernelGGL(text_embed_kernel, dim3(ceil_div(te, 256)), dim3(256), 0, s, x, tokens, prompts, w->tok_emb,
                       w->pos_emb, N, L, Lt, W, (int64_t)w->vocab);
    RM_LAUNCHED();
    int rc;
    for (int i = 0; i < w->layers; i++) {
        const reidmi_block_weights& bw = w->blocks[i];
        if (i > 0 && bw.prompt && w->n_ctx > 0) {
            const int64_t pe = N * w->n_ctx * W;
            hipLaunchKernelGGL(prompt_rows_kernel, dim3(ceil_div(pe, 256)), dim3(256), 0, s, x, N, L, W, 1,
                               w->n_ctx, bw.prompt);
            RM_LAUNCHED();
        }
        const XStats xs = i > 0 && !(bw.prompt && w->n_ctx > 0) ? XS_PARTIALS : XS_ROWS;
        if ((rc = run_block(bw, ws, P, N, L, W, w->heads, true, xs, s))) return rc;
    }
    hipLaunchKernelGGL(eot_rows_kernel, dim3(ceil_div(N, 256)), dim3(256), 0, s, tokens, N, L, Lt, rows);
    RM_LAUNCHED();
    if ((rc = layernorm(x, N, W, rows, W, w->ln_final_w, w->ln_final_b, 1e-5f, nullptr, 0, h, W, s))) return rc;
    EpiArgs eo{};
    eo.out = out;
    eo.ldc = E;
    return gemm_f16(EPI_F32, h, W, w->proj_t, W, N, E, W, eo, s);
}

// LayerNorm row statistics as the encoder computes them (test entry points): st[r] =
// (rstd, -mean * rstd) of the fp16 rows x, from a pass over x (pst == NULL) or combined from
// the residual epilogue's 64-column partials pst [W/64][rows] (run_block's ln_1 / ln_2).
REIDMI_API int reidmi_row_stats_f16(const void* x, int64_t rows, int64_t ldx, int64_t W, const void* pst, void* st,
                                    void* stream) {
    RM_REQUIRE(st && (x || pst), "row stats: null argument");
    if (pst) return row_stats_from_partials((const float2*)pst, rows, (int)W, (float2*)st, (hipStream_t)stream);
    return row_stats((const _Float16*)x, rows, ldx, W, (float2*)st, (hipStream_t)stream);
}

// The residual GEMM of run_block with its LayerNorm partials: out[m][n] = half(out[m][n] +
// (A W^T)[m][n] + bias[n]) and pst[n/64 * M + m] = (sum, centred sum of squares) of the 64
// updated values of row m in column block n/64 (N % 64 == 0).
REIDMI_API int reidmi_gemm_f16_resid_partials(const void* A, int64_t lda, const void* Wt, int64_t ldw, int64_t M,
                                              int64_t N, int64_t K, const float* bias, void* out, int64_t ldc,
                                              void* pst, void* stream) {
    RM_REQUIRE(A && Wt && out && pst && N % 64 == 0, "resid partials: null argument or N % 64 != 0");
    EpiArgs e{};
    e.out = out;
    e.ldc = ldc;
    e.bias = bias;
    e.pstat = (float2*)pst;
    e.ldp = M;
    return gemm_f16(EPI_RESID_F16, (const _Float16*)A, lda, (const _Float16*)Wt, ldw, M, (int)N, (int)K, e,
                    (hipStream_t)stream);
}

#ifdef REIDMI_TOOLS
// ln_1-folded QKV projection + attention of one block (custom_clip_model.py:22-27) on its own,
// for tests / A-B timing (tools library, include/reidmi_tools.h): fused = 1 the single fused kernel, 0 the QKV GEMM (head-split
// epilogue into q, k [nseq*H][L][64], vt [nseq*H][64][reidmi_attn_lpad(L)]) then the attention
// kernel.  The two are bit-identical (same MFMA chains, same roundings).
REIDMI_API int reidmi_qkv_attention_f16(const void* x, int64_t ldx, const void* wq, int64_t ldw, const float* bias,
                                        const float* colsum, const void* rowstat, int64_t nseq, int L, int H, int W,
                                        void* q, void* k, void* vt, void* o, int fused, void* stream) {
    hipStream_t s = (hipStream_t)stream;
    RM_REQUIRE(W == H * 64 && L > 0 && nseq >= 0 && rowstat && colsum && bias, "qkv_attention: bad arguments");
    if (fused) {
        RM_REQUIRE(qkv_attn_fits(L, W, false), "qkv_attention: the fused kernel takes 192 < L <= 224 tokens");
        return qkv_attn(x, ldx, wq, ldw, bias, colsum, rowstat, nseq, L, H, W, o, s);
    }
    RM_REQUIRE(q && k && vt, "qkv_attention: q / k / vt scratch required for the unfused path");
    EpiArgs ea{};
    ea.bias = bias;
    ea.rowstat = (const float2*)rowstat;
    ea.colsum = colsum;
    ea.q = q;
    ea.k = k;
    ea.vt = vt;
    ea.seq = L;
    ea.heads = H;
    ea.lpad = attn_lpad(L);
    int rc;
    if ((rc = gemm_f16(EPI_QKV, x, ldx, wq, ldw, nseq * L, 3 * W, W, ea, s))) return rc;
    return mhsa(q, k, vt, o, nseq, L, H, false, s);
}
#endif  // REIDMI_TOOLS
