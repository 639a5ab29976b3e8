// pack.hip — weight packing for the encoders (reidmi_vit_weights_pack / reidmi_text_weights_pack).
//
// The checkpoint boundary of SURVEY.md §8b: a caller holding the reference's fp32 tensors on the
// device, in the reference's key layout (utils.py:169-221: CLIP-ReID `image_encoder.*` keys ->
// custom_clip_model.VisionTransformer, custom_clip_model.py:57-100; zero_shot_learning.py:28-35:
// `text_encoder.*` keys -> the CLIP text tower, maple.py:971-984), gets a runnable
// reidmi_vit_weights / reidmi_text_weights whose device data all lives in one caller-owned buffer.
// What the packing computes (load time; the same definitions as multimodal_reid_amd.model):
//   * ln_1 / ln_2 folded into the GEMM they feed (gemm.h EpiArgs): W' = fp16(W diag(gamma)) with the
//     product rounded to fp32 first and then to fp16 (exactly what torch's fp64 -> fp16 cast does:
//     it goes through fp32, and the fp32 x fp32 product is exact in fp64), s_n = sum_k W'[n, k]
//     (exact: 768-1024 fp16 values sum without rounding in fp64), b' = fp32(b + sum_k W[n, k] beta_k)
//     with the products exact in fp64 and the sum compensated (TwoSum), i.e. correctly rounded
//     except for astronomically rare ties;
//   * the other matrices cast to fp16 (the reference's GPU dtype, utils.py:145-166 convert_weights);
//     conv1 flattened (c, ky, kx) and zero-padded to a multiple of 64; proj / text_projection
//     transposed ([out][in], the GEMM's W^T operand);
//   * every fp32 vector (LayerNorms, biases, embeddings, VPT prompts) copied as is.
// Stream-ordered, no allocation, no synchronisation.
#include "common.h"

namespace reidmi {

// (s, c) += x with Neumaier/TwoSum compensation
__device__ __forceinline__ void two_sum_acc(double& s, double& c, double x) {
    const double t = s + x;
    const double bp = t - s;
    const double e = (s - (t - bp)) + (x - bp);
    s = t;
    c += e;
}

// One wave per output row n of a LayerNorm-folded Linear: wf[n][:] (fp16), colsum[n], bias'[n].
__global__ __launch_bounds__(256) void fold_rows_kernel(const float* __restrict__ w, int64_t N, int K,
                                                        const float* __restrict__ b, const float* __restrict__ gamma,
                                                        const float* __restrict__ beta, _Float16* __restrict__ wf,
                                                        float* __restrict__ colsum, float* __restrict__ bias) {
    const int lane = threadIdx.x & 63;
    const int64_t n = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (n >= N) return;
    const float* wr = w + n * K;
    _Float16* hr = wf + n * K;
    double cs = 0.0, s = 0.0, c = 0.0;
    for (int k = lane; k < K; k += 64) {
        const float wk = wr[k];
        float p = wk * gamma[k];  // fp32 product (= the exact fp64 product rounded to fp32) ...
        // ... then fp16 RNE: two roundings, as torch's fp64 -> fp16 cast.  The opaque copy keeps
        // the backend from merging the multiply and the conversion into one v_fma_mix (one
        // rounding), as it did in the attention epilogue.
        asm volatile("" : "+v"(p));
        const _Float16 h = (_Float16)p;
        hr[k] = h;
        cs += (double)h;  // exact
        two_sum_acc(s, c, (double)wk * (double)beta[k]);  // product exact in fp64
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        cs += __shfl_xor(cs, o, 64);
        const double s2 = __shfl_xor(s, o, 64), c2 = __shfl_xor(c, o, 64);
        two_sum_acc(s, c, s2);
        c += c2;
    }
    if (lane == 0) {
        two_sum_acc(s, c, (double)b[n]);
        colsum[n] = (float)cs;
        bias[n] = (float)(s + c);
    }
}

// fp32 [rows][cols] (row stride lds) -> fp16 [rows][ldd], columns >= cols zero (ldd >= cols)
__global__ __launch_bounds__(256) void cast_pad_f16_kernel(const float* __restrict__ src, int64_t rows, int64_t cols,
                                                           int64_t lds, _Float16* __restrict__ dst, int64_t ldd) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= rows * ldd) return;
    const int64_t r = t / ldd, cidx = t - r * ldd;
    dst[t] = cidx < cols ? (_Float16)src[r * lds + cidx] : (_Float16)0.0f;
}

// fp32 [rows][cols] -> fp16 transposed [cols][rows] (32 x 32 tiles through LDS)
__global__ __launch_bounds__(256) void transpose_f16_kernel(const float* __restrict__ src, int64_t rows, int64_t cols,
                                                            _Float16* __restrict__ dst) {
    __shared__ float tile[32][33];
    const int64_t r0 = (int64_t)blockIdx.y * 32, c0 = (int64_t)blockIdx.x * 32;
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
    for (int i = ty; i < 32; i += 8) {
        const int64_t r = r0 + i, cidx = c0 + tx;
        tile[i][tx] = (r < rows && cidx < cols) ? src[r * cols + cidx] : 0.f;
    }
    __syncthreads();
    for (int i = ty; i < 32; i += 8) {
        const int64_t cidx = c0 + i, r = r0 + tx;
        if (cidx < cols && r < rows) dst[cidx * rows + r] = (_Float16)tile[tx][i];
    }
}

namespace {

constexpr int64_t kAlign = 256;

struct Arena {  // offsets first (base == nullptr: sizing pass), then pointers
    char* base;
    int64_t off = 0;
    template <typename T>
    T* take(int64_t n) {
        off = (off + kAlign - 1) / kAlign * kAlign;
        T* p = base ? (T*)(base + off) : nullptr;
        off += n * (int64_t)sizeof(T);
        return p;
    }
};

int copy_f32(Arena& a, const float* src, int64_t n, const float** dst, hipStream_t s) {
    float* d = a.take<float>(n);
    if (a.base) {
        RM_REQUIRE(src != nullptr, "weights_pack: a required fp32 tensor is NULL");
        RM_CHECK_HIP(hipMemcpyAsync(d, src, n * sizeof(float), hipMemcpyDeviceToDevice, s));
    }
    *dst = d;
    return OK;
}

int cast_f16(Arena& a, const float* src, int64_t rows, int64_t cols, int64_t ldd, const void** dst, hipStream_t s) {
    _Float16* d = a.take<_Float16>(rows * ldd);
    if (a.base) {
        RM_REQUIRE(src != nullptr, "weights_pack: a required matrix is NULL");
        const int64_t n = rows * ldd;
        hipLaunchKernelGGL(cast_pad_f16_kernel, dim3(ceil_div(n, 256)), dim3(256), 0, s, src, rows, cols, cols, d, ldd);
        RM_LAUNCHED();
    }
    *dst = d;
    return OK;
}

int transpose_f16(Arena& a, const float* src, int64_t rows, int64_t cols, const void** dst, hipStream_t s) {
    _Float16* d = a.take<_Float16>(rows * cols);
    if (a.base) {
        RM_REQUIRE(src != nullptr, "weights_pack: a projection matrix is NULL");
        hipLaunchKernelGGL(transpose_f16_kernel, dim3(ceil_div(cols, 32), ceil_div(rows, 32)), dim3(256), 0, s, src,
                           rows, cols, d);
        RM_LAUNCHED();
    }
    *dst = d;
    return OK;
}

int fold(Arena& a, const float* w, const float* b, const float* g, const float* be, int64_t N, int K, const void** wf,
         const float** bf, const float** cs, hipStream_t s) {
    _Float16* dw = a.take<_Float16>(N * K);
    float* dc = a.take<float>(N);
    float* db = a.take<float>(N);
    if (a.base) {
        RM_REQUIRE(w && b && g && be, "weights_pack: a LayerNorm-folded Linear needs weight, bias, gamma, beta");
        hipLaunchKernelGGL(fold_rows_kernel, dim3(ceil_div(N, 4)), dim3(256), 0, s, w, N, K, b, g, be, dw, dc, db);
        RM_LAUNCHED();
    }
    *wf = dw;
    *cs = dc;
    *bf = db;
    return OK;
}

int pack_blocks(Arena& a, const reidmi_block_src* src, int layers, int W, int n_ctx, reidmi_block_weights* out,
                hipStream_t s) {
    int rc;
    for (int i = 0; i < layers; i++) {
        const reidmi_block_src& b = src[i];
        reidmi_block_weights& o = out[i];
        if ((rc = copy_f32(a, b.ln_1_w, W, &o.ln1_w, s)) || (rc = copy_f32(a, b.ln_1_b, W, &o.ln1_b, s)) ||
            (rc = fold(a, b.in_proj_w, b.in_proj_b, b.ln_1_w, b.ln_1_b, 3 * (int64_t)W, W, &o.qkv_w, &o.qkv_b,
                       &o.qkv_s, s)) ||
            (rc = cast_f16(a, b.out_proj_w, W, W, W, &o.out_w, s)) || (rc = copy_f32(a, b.out_proj_b, W, &o.out_b, s)) ||
            (rc = copy_f32(a, b.ln_2_w, W, &o.ln2_w, s)) || (rc = copy_f32(a, b.ln_2_b, W, &o.ln2_b, s)) ||
            (rc = fold(a, b.c_fc_w, b.c_fc_b, b.ln_2_w, b.ln_2_b, 4 * (int64_t)W, W, &o.fc1_w, &o.fc1_b, &o.fc1_s,
                       s)) ||
            (rc = cast_f16(a, b.c_proj_w, W, 4 * (int64_t)W, 4 * (int64_t)W, &o.fc2_w, s)) ||
            (rc = copy_f32(a, b.c_proj_b, W, &o.fc2_b, s)))
            return rc;
        o.prompt = nullptr;
        if (b.vpt_shallow && n_ctx > 0) {
            if ((rc = copy_f32(a, b.vpt_shallow, (int64_t)n_ctx * W, &o.prompt, s))) return rc;
        }
    }
    return OK;
}

int vit_src_check(const reidmi_vit_src* s) {
    RM_REQUIRE(s && s->blocks, "vit_weights_pack: null source");
    RM_REQUIRE(s->width > 0 && s->width % 256 == 0 && s->layers >= 12 && s->patch > 0 && s->stride > 0 &&
                   s->out_dim > 0 && s->out_dim % 128 == 0 && s->grid_h > 0 && s->grid_w > 0 && s->n_ctx >= 0,
               "vit_weights_pack: width % 256 == 0, layers >= 12 (resblocks[:12] run), out_dim % 128 == 0, "
               "positive patch / stride / grid");
    return OK;
}

int text_src_check(const reidmi_text_src* s) {
    RM_REQUIRE(s && s->blocks, "text_weights_pack: null source");
    RM_REQUIRE(s->width > 0 && s->width % 256 == 0 && s->layers > 0 && s->ctx > 0 && s->ctx <= 256 && s->vocab > 0 &&
                   s->out_dim > 0 && s->out_dim % 128 == 0 && s->n_ctx >= 0,
               "text_weights_pack: width % 256 == 0, 0 < ctx <= 256, out_dim % 128 == 0");
    return OK;
}

int vit_pack(const reidmi_vit_src* src, char* buf, int64_t* bytes, reidmi_vit_weights* w, reidmi_block_weights* blocks,
             hipStream_t s) {
    int rc;
    if ((rc = vit_src_check(src))) return rc;
    Arena a{buf};
    const int W = src->width, P = src->patch, E = src->out_dim;
    const int kpad = (3 * P * P + 63) / 64 * 64;
    const int64_t npos = 1 + (int64_t)src->grid_h * src->grid_w;
    reidmi_vit_weights tmp{};
    tmp.width = W;
    tmp.layers = src->layers;
    tmp.heads = W / 64;
    tmp.patch = P;
    tmp.stride = src->stride;
    tmp.out_dim = E;
    tmp.grid_h = src->grid_h;
    tmp.grid_w = src->grid_w;
    tmp.n_ctx = src->n_ctx;
    tmp.kpad = kpad;
    if ((rc = cast_f16(a, src->conv1_w, W, 3 * P * P, kpad, &tmp.conv_w, s)) ||
        (rc = copy_f32(a, src->class_embedding, W, &tmp.class_emb, s)) ||
        (rc = copy_f32(a, src->positional_embedding, npos * W, &tmp.pos_emb, s)) ||
        (rc = copy_f32(a, src->ln_pre_w, W, &tmp.ln_pre_w, s)) || (rc = copy_f32(a, src->ln_pre_b, W, &tmp.ln_pre_b, s)) ||
        (rc = copy_f32(a, src->ln_post_w, W, &tmp.ln_post_w, s)) ||
        (rc = copy_f32(a, src->ln_post_b, W, &tmp.ln_post_b, s)) ||
        (rc = transpose_f16(a, src->proj, W, E, &tmp.proj_t, s)))
        return rc;
    tmp.vpt = nullptr;
    if (src->n_ctx > 0) {
        RM_REQUIRE(src->vpt != nullptr, "vit_weights_pack: n_ctx > 0 needs VPT");
        if ((rc = copy_f32(a, src->vpt, (int64_t)src->n_ctx * W, &tmp.vpt, s))) return rc;
    }
    if (buf) {
        RM_REQUIRE(blocks != nullptr && w != nullptr, "vit_weights_pack: out / out_blocks required");
    }
    // sizing pass: block pointers go to a scratch array
    reidmi_block_weights* bo = blocks;
    reidmi_block_weights dummy[1];
    for (int i = 0; i < src->layers; i++) {
        if ((rc = pack_blocks(a, src->blocks + i, 1, W, src->n_ctx, bo ? bo + i : dummy, s))) return rc;
    }
    *bytes = a.off;
    if (w) {
        tmp.blocks = blocks;
        *w = tmp;
    }
    return OK;
}

int text_pack(const reidmi_text_src* src, char* buf, int64_t* bytes, reidmi_text_weights* w,
              reidmi_block_weights* blocks, hipStream_t s) {
    int rc;
    if ((rc = text_src_check(src))) return rc;
    Arena a{buf};
    const int W = src->width, E = src->out_dim;
    reidmi_text_weights tmp{};
    tmp.width = W;
    tmp.layers = src->layers;
    tmp.heads = W / 64;
    tmp.ctx = src->ctx;
    tmp.vocab = src->vocab;
    tmp.out_dim = E;
    tmp.n_ctx = src->n_ctx;
    if ((rc = copy_f32(a, src->token_embedding, (int64_t)src->vocab * W, &tmp.tok_emb, s)) ||
        (rc = copy_f32(a, src->positional_embedding, (int64_t)src->ctx * W, &tmp.pos_emb, s)) ||
        (rc = copy_f32(a, src->ln_final_w, W, &tmp.ln_final_w, s)) ||
        (rc = copy_f32(a, src->ln_final_b, W, &tmp.ln_final_b, s)) ||
        (rc = transpose_f16(a, src->text_projection, W, E, &tmp.proj_t, s)))
        return rc;
    if (buf) {
        RM_REQUIRE(blocks != nullptr && w != nullptr, "text_weights_pack: out / out_blocks required");
    }
    reidmi_block_weights dummy[1];
    for (int i = 0; i < src->layers; i++) {
        if ((rc = pack_blocks(a, src->blocks + i, 1, W, src->n_ctx, blocks ? blocks + i : dummy, s))) return rc;
    }
    *bytes = a.off;
    if (w) {
        tmp.blocks = blocks;
        *w = tmp;
    }
    return OK;
}

}  // namespace
}  // namespace reidmi

using namespace reidmi;

REIDMI_API int64_t reidmi_vit_pack_bytes(const reidmi_vit_src* src) {
    int64_t n = 0;
    return vit_pack(src, nullptr, &n, nullptr, nullptr, nullptr) ? -1 : n;
}

REIDMI_API int reidmi_vit_weights_pack(const reidmi_vit_src* src, void* buf, int64_t buf_bytes, reidmi_vit_weights* out,
                                       reidmi_block_weights* out_blocks, void* stream) {
    int64_t n = 0;
    int rc;
    if ((rc = vit_pack(src, nullptr, &n, nullptr, nullptr, nullptr))) return rc;
    RM_REQUIRE(buf != nullptr && buf_bytes >= n && ((uintptr_t)buf & (kAlign - 1)) == 0,
               "vit_weights_pack: buffer smaller than reidmi_vit_pack_bytes or not 256-byte aligned");
    return vit_pack(src, (char*)buf, &n, out, out_blocks, (hipStream_t)stream);
}

REIDMI_API int64_t reidmi_text_pack_bytes(const reidmi_text_src* src) {
    int64_t n = 0;
    return text_pack(src, nullptr, &n, nullptr, nullptr, nullptr) ? -1 : n;
}

REIDMI_API int reidmi_text_weights_pack(const reidmi_text_src* src, void* buf, int64_t buf_bytes,
                                        reidmi_text_weights* out, reidmi_block_weights* out_blocks, void* stream) {
    int64_t n = 0;
    int rc;
    if ((rc = text_pack(src, nullptr, &n, nullptr, nullptr, nullptr))) return rc;
    RM_REQUIRE(buf != nullptr && buf_bytes >= n && ((uintptr_t)buf & (kAlign - 1)) == 0,
               "text_weights_pack: buffer smaller than reidmi_text_pack_bytes or not 256-byte aligned");
    return text_pack(src, (char*)buf, &n, out, out_blocks, (hipStream_t)stream);
}
