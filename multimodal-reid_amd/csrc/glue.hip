// glue.hip — the per-image feature epilogue of zero_shot_learning.inference (G1).
//
// Non-multimodal (zero_shot_learning.py:93,124-126):
//     emb = (cat(x12[:,0], xproj[:,0]) + cat(x12'[:,0], xproj'[:,0])) / 2
// Multimodal --mm (zero_shot_learning.py:95-97,116-122):
//     p = normalize((xproj[:,0] + xproj'[:,0]) / 2)
//     emb = cat((x12[:,0] + x12'[:,0]) / 2, softmax((1/0.07) * p @ zeroshot_weights^T))
// (primed = the augmented-loader pass).  Computed in fp32 on the GPU right after the two
// encoder passes, so features never leave HBM before the distance stage.
#include "common.h"

namespace reidmi {

__global__ void tta_avg_kernel(const float* __restrict__ x12a, const float* __restrict__ pa,
                               const float* __restrict__ x12b, const float* __restrict__ pb, int64_t B, int64_t W,
                               int64_t E, float* __restrict__ emb, int64_t lde) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t D = W + E;
    if (e >= B * D) return;
    const int64_t b = e / D, c = e % D;
    const float v = c < W ? (x12a[b * W + c] + x12b[b * W + c]) : (pa[b * E + c - W] + pb[b * E + c - W]);
    emb[b * lde + c] = v / 2.0f;
}

__device__ float block_sum(float v, float* red) {
    v = wave_sum(v);
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    float t = 0.f;
    for (int i = 0; i < (int)(blockDim.x >> 6); i++) t += red[i];
    return t;
}
__device__ float block_max(float v, float* red) {
    v = wave_max(v);
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    float t = -__builtin_inff();
    for (int i = 0; i < (int)(blockDim.x >> 6); i++) t = fmaxf(t, red[i]);
    return t;
}

// one 256-thread workgroup per image; dynamic LDS: E floats (p) + ncls floats (logits)
__global__ __launch_bounds__(256) void tta_mm_kernel(const float* __restrict__ x12a, const float* __restrict__ pa,
                                                     const float* __restrict__ x12b, const float* __restrict__ pb,
                                                     const float* __restrict__ zs, int64_t W, int64_t E,
                                                     int64_t ncls, float* __restrict__ emb, int64_t lde) {
    extern __shared__ float sm[];
    __shared__ float red[8];
    float* p = sm;
    float* lg = sm + E;
    const int64_t b = blockIdx.x;
    for (int64_t c = threadIdx.x; c < W; c += blockDim.x)
        emb[b * lde + c] = (x12a[b * W + c] + x12b[b * W + c]) / 2.0f;
    float ss = 0.f;
    for (int64_t c = threadIdx.x; c < E; c += blockDim.x) {
        const float v = (pa[b * E + c] + pb[b * E + c]) / 2.0f;
        p[c] = v;
        ss += v * v;
    }
    const float nrm = __builtin_sqrtf(block_sum(ss, red));
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    for (int64_t c = wid; c < ncls; c += 4) {
        const float* z = zs + c * E;
        float d = 0.f;
        for (int64_t k = lane; k < E; k += 64) d += p[k] * z[k];
        d = wave_sum(d);
        if (lane == 0) lg[c] = (1.0f / 0.07f) * (d / nrm);
    }
    __syncthreads();
    float mx = -__builtin_inff();
    for (int64_t c = threadIdx.x; c < ncls; c += blockDim.x) mx = fmaxf(mx, lg[c]);
    mx = block_max(mx, red);
    float se = 0.f;
    for (int64_t c = threadIdx.x; c < ncls; c += blockDim.x) {
        const float ex = __expf(lg[c] - mx);
        lg[c] = ex;
        se += ex;
    }
    se = block_sum(se, red);
    for (int64_t c = threadIdx.x; c < ncls; c += blockDim.x) emb[b * lde + W + c] = lg[c] / se;
}

// zeroshot_classifier (zero_shot_learning.py:42-48): per class c with template rows
// [off[c], off[c+1]): normalise each row, mean over rows, normalise.  One workgroup per class.
__global__ __launch_bounds__(256) void class_mean_norm_kernel(const float* __restrict__ f, const int64_t* __restrict__ off,
                                                              int64_t E, float* __restrict__ out) {
    extern __shared__ float acc[];
    __shared__ float red[8];
    const int64_t c = blockIdx.x;
    for (int64_t k = threadIdx.x; k < E; k += blockDim.x) acc[k] = 0.f;
    const int64_t r0 = off[c], r1 = off[c + 1];
    for (int64_t r = r0; r < r1; r++) {
        float ss = 0.f;
        for (int64_t k = threadIdx.x; k < E; k += blockDim.x) ss += f[r * E + k] * f[r * E + k];
        const float inv = 1.0f / __builtin_sqrtf(block_sum(ss, red));
        for (int64_t k = threadIdx.x; k < E; k += blockDim.x) acc[k] += f[r * E + k] * inv;
    }
    const float n = (float)(r1 - r0);
    float ss = 0.f;
    for (int64_t k = threadIdx.x; k < E; k += blockDim.x) {
        acc[k] = acc[k] / n;
        ss += acc[k] * acc[k];
    }
    const float inv = 1.0f / __builtin_sqrtf(block_sum(ss, red));
    for (int64_t k = threadIdx.x; k < E; k += blockDim.x) out[c * E + k] = acc[k] * inv;
}

// Prompt construction (T3): coop.PromptLearner.forward (coop.py:95-110) and
// maple.VLPromptLearner.construct_prompts (maple.py:57-90): for each label b,
// prompts[b] = cat(prefix [P][W], ctx[label[b]] [C][W], suffix [S][W]) along the tokens.
// One float4 per thread; prefix / suffix rows are shared by every label.
__global__ void prompt_build_kernel(const float* __restrict__ prefix, int P, const float* __restrict__ ctx, int C,
                                    const int64_t* __restrict__ label, int64_t ncls, const float* __restrict__ suffix,
                                    int S, int64_t B, int W, float* __restrict__ out, int32_t* __restrict__ bad) {
    const int L = P + C + S, W4 = W / 4;
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= B * L * W4) return;
    const int c4 = (int)(e % W4);
    const int64_t bt = e / W4;
    const int t = (int)(bt % L);
    const int64_t b = bt / L;
    const float* src;
    if (t < P) src = prefix + (int64_t)t * W;
    else if (t < P + C) {
        int64_t lb = label[b];
        if (lb < 0 || lb >= ncls) {  // an out-of-range label: flagged, row 0 used
            if (bad) *bad = 1;
            lb = 0;
        }
        src = ctx + (lb * C + (t - P)) * (int64_t)W;
    } else src = suffix + (int64_t)(t - P - C) * W;
    ((float4*)(out + bt * W))[c4] = ((const float4*)src)[c4];
}

}  // namespace reidmi

using namespace reidmi;

REIDMI_API int reidmi_prompt_build(const float* prefix, int P, const float* ctx, int C, const int64_t* label,
                                   int64_t ncls, const float* suffix, int S, int64_t B, int W, float* out,
                                   int32_t* bad_label, void* stream) {
    RM_REQUIRE(P >= 0 && C >= 0 && S >= 0 && P + C + S > 0 && B >= 0 && W > 0 && W % 4 == 0 && ncls > 0,
               "prompt_build: bad shape");
    if (B == 0) return OK;
    const int64_t n = B * (P + C + S) * (W / 4);
    hipLaunchKernelGGL(prompt_build_kernel, dim3(ceil_div(n, 256)), dim3(256), 0, (hipStream_t)stream, prefix, P, ctx,
                       C, label, ncls, suffix, S, B, W, out, bad_label);
    RM_LAUNCHED();
    return OK;
}

REIDMI_API int reidmi_class_mean_normalize(const float* feats, const int64_t* offsets, int64_t ncls, int64_t E,
                                           float* out, void* stream) {
    RM_REQUIRE(ncls >= 0 && E > 0 && E * 4 <= 64 * 1024, "class_mean_normalize: bad shape");
    if (ncls == 0) return OK;
    hipLaunchKernelGGL(class_mean_norm_kernel, dim3((unsigned)ncls), dim3(256), E * 4, (hipStream_t)stream, feats,
                       offsets, E, out);
    RM_LAUNCHED();
    return OK;
}

REIDMI_API int reidmi_feature_tta_avg(const float* x12a, const float* pa, const float* x12b, const float* pb,
                                      int64_t B, int64_t W, int64_t E, float* emb, int64_t lde, void* stream) {
    RM_REQUIRE(B >= 0 && W > 0 && E > 0 && lde >= W + E, "feature_tta_avg: bad shape");
    if (B == 0) return OK;
    hipLaunchKernelGGL(tta_avg_kernel, dim3(ceil_div(B * (W + E), 256)), dim3(256), 0, (hipStream_t)stream, x12a, pa,
                       x12b, pb, B, W, E, emb, lde);
    RM_LAUNCHED();
    return OK;
}

REIDMI_API int reidmi_feature_tta_mm(const float* x12a, const float* pa, const float* x12b, const float* pb,
                                     const float* zs, int64_t B, int64_t W, int64_t E, int64_t ncls, float* emb,
                                     int64_t lde, void* stream) {
    RM_REQUIRE(B >= 0 && W > 0 && E > 0 && ncls > 0 && lde >= W + ncls, "feature_tta_mm: bad shape");
    const size_t lds = (size_t)(E + ncls) * 4;
    RM_REQUIRE(lds <= 64 * 1024, "feature_tta_mm: E + ncls too large");
    if (B == 0) return OK;
    hipLaunchKernelGGL(tta_mm_kernel, dim3((unsigned)B), dim3(256), lds, (hipStream_t)stream, x12a, pa, x12b, pb, zs,
                       W, E, ncls, emb, lde);
    RM_LAUNCHED();
    return OK;
}
