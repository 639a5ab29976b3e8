// transforms.hip — the reference's test-time image transform on the GPU:
//   transforms.Resize((oh, ow)) -> ToTensor() -> Normalize(mean, std)   (data_prepare.py:257-261)
// applied to decoded RGB images (data_prepare.py:88).  torchvision hands a PIL image to
// PIL.Image.resize((ow, oh), BILINEAR), so the arithmetic reproduced here, bit for bit, is
// Pillow's 8-bit separable resampler (restated and pinned against Pillow 12.2 in
// oracle/transforms_oracle.c): per-axis triangle-filter coefficients computed in double and
// rounded to 22-bit fixed point, a horizontal then a vertical integer pass (vertical first
// for tall narrow sources, h > 100 w), each output clip8((2^21 + sum k_i p_i) >> 22).
// The flip / pad / crop of the TTA loader (data_prepare.py:263-270) commute with ToTensor
// and Normalize and are applied by the encoder's im2col (encoder.hip) on these outputs.
//
// Layout: the batch arrives packed (concatenated HWC uint8 images + per-image (byte offset,
// h, w)); JPEG decode stays on the host.  One workgroup per (image, band of 32 output rows):
// the band's coefficient rows and its first-pass intermediate (source rows the band reads
// x ow x 3 bytes) live in LDS, so every source byte is read from L2 a few times and every
// output element is written once, coalesced along x.  Integer work, HBM-bound on the
// output writes (3 * oh * ow * 4 or 2 bytes per image).
#include "common.h"

namespace reidmi {

constexpr int PP_BAND = 32;   // output rows per workgroup
constexpr int PP_PREC = 22;   // Pillow PRECISION_BITS = 32 - 8 - 2

__device__ __forceinline__ double pp_tri(double x) {
    if (x < 0.0) x = -x;
    if (x < 1.0) return 1.0 - x;
    return 0.0;
}

__host__ __device__ __forceinline__ int pp_ksize(int in, int out) {
    const double scale = (double)in / out;
    const double support = scale < 1.0 ? 1.0 : scale;
    return (int)ceil(support) * 2 + 1;
}

// Pillow precompute_coeffs + normalize_coeffs_8bpc for output index o (one thread).
__device__ void pp_coeffs(int in, int out, int o, int ksize, int* bnd, int* kk) {
    const double scale = (double)in / out;
    const double fs = scale < 1.0 ? 1.0 : scale;
    const double support = 1.0 * fs;
    const double center = 0.0 + (o + 0.5) * scale;
    const double ss = 1.0 / fs;
    int xmin = (int)(center - support + 0.5);
    if (xmin < 0) xmin = 0;
    int xmax = (int)(center + support + 0.5);
    if (xmax > in) xmax = in;
    xmax -= xmin;
    double ww = 0.0;
    for (int i = 0; i < xmax; i++) ww += pp_tri((i + xmin - center + 0.5) * ss);
    for (int i = 0; i < ksize; i++) {
        double w = 0.0;
        if (i < xmax) {
            w = pp_tri((i + xmin - center + 0.5) * ss);
            if (ww != 0.0) w /= ww;
        }
        kk[i] = w < 0 ? (int)(-0.5 + w * (1 << PP_PREC)) : (int)(0.5 + w * (1 << PP_PREC));
    }
    bnd[0] = xmin;
    bnd[1] = xmax;
}

__device__ __forceinline__ uint8_t pp_clip8(int v) {
    v >>= PP_PREC;
    return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
}

struct PPArgs {
    const uint8_t* pix;
    const int64_t* meta;  // [B][3] (byte offset, h, w)
    int oh, ow;
    int max_h, max_w;
    int kh_cap, kv_cap, rows_cap;
    float mean[3], stdv[3];
    int out_f16;
    void* out;
};

__global__ __launch_bounds__(256) void preprocess_kernel(PPArgs a) {
    extern __shared__ __attribute__((aligned(16))) int pp_lds[];
    const int b = blockIdx.y;
    const int y_lo = blockIdx.x * PP_BAND;
    const int oh = a.oh, ow = a.ow;
    const int y_hi = min(y_lo + PP_BAND, oh), nb = y_hi - y_lo;
    const int64_t off = a.meta[3 * b];
    const int h = (int)a.meta[3 * b + 1], w = (int)a.meta[3 * b + 2];
    if (h <= 0 || w <= 0 || h > a.max_h || w > a.max_w) return;  // caller contract (reidmi.h)
    const uint8_t* src = a.pix + off;
    const bool need_h = ow != w, need_v = oh != h;
    const bool vfirst = need_h && need_v && oh < h && (int64_t)h > 100 * (int64_t)w;
    const int KH = pp_ksize(w, ow), KV = pp_ksize(h, oh);

    // LDS: normalise LUT [3][256] f32 | h bounds [ow][2] | h coeffs [ow][kh_cap] |
    //      v bounds [BAND][2] | v coeffs [BAND][kv_cap] | intermediate bytes
    float* lut = (float*)pp_lds;
    int* hb = pp_lds + 768;
    int* hk = hb + 2 * ow;
    int* vb = hk + ow * a.kh_cap;
    int* vk = vb + 2 * PP_BAND;
    uint8_t* mid = (uint8_t*)(vk + PP_BAND * a.kv_cap);
    const int tid = threadIdx.x;

    for (int i = tid; i < 768; i += 256) {
        const int c = i >> 8, p = i & 255;
        const float v = (float)p / 255.0f;  // ToTensor (correctly rounded division)
        lut[i] = (v - a.mean[c]) / a.stdv[c];  // Normalize
    }
    if (need_h)
        for (int o = tid; o < ow; o += 256) pp_coeffs(w, ow, o, KH, hb + 2 * o, hk + o * KH);
    if (need_v)
        for (int o = tid; o < nb; o += 256) pp_coeffs(h, oh, y_lo + o, KV, vb + 2 * o, vk + o * KV);
    __syncthreads();

    const int64_t plane = (int64_t)oh * ow;
    // 4 consecutive outputs x..x+3 of channel c, row yi (ow % 4 == 0: 8- or 16-byte stores)
    auto emit4 = [&](int yi, int x, int c, const uint8_t (&p)[4][3]) {
        const int64_t e = ((int64_t)b * 3 + c) * plane + (int64_t)(y_lo + yi) * ow + x;
        const float v0 = lut[c * 256 + p[0][c]], v1 = lut[c * 256 + p[1][c]];
        const float v2 = lut[c * 256 + p[2][c]], v3 = lut[c * 256 + p[3][c]];
        if (a.out_f16)
            *(u16x4*)((unsigned short*)a.out + e) = u16x4{f2h_bits(v0), f2h_bits(v1), f2h_bits(v2), f2h_bits(v3)};
        else
            *(float4*)((float*)a.out + e) = make_float4(v0, v1, v2, v3);
    };

    if (!vfirst) {
        // first pass: horizontal over the source rows the band reads -> mid[r - r0][x][c]
        int r0 = y_lo, r1 = y_hi;
        if (need_v) {
            r0 = vb[0];
            r1 = vb[2 * (nb - 1)] + vb[2 * (nb - 1) + 1];
        }
        if (r1 - r0 > a.rows_cap) r1 = r0 + a.rows_cap;  // unreachable by the host-side bound
        const int tw = need_h ? ow : w;  // == ow
        for (int it = tid; it < (r1 - r0) * tw; it += 256) {
            const int r = r0 + it / tw, x = it % tw;
            const uint8_t* row = src + (int64_t)r * w * 3;
            uint8_t* m = mid + (int64_t)it * 3;
            if (need_h) {
                const int x0 = hb[2 * x], n = hb[2 * x + 1];
                const int* k = hk + x * KH;
                int s0 = 1 << (PP_PREC - 1), s1 = s0, s2 = s0;
                for (int i = 0; i < n; i++) {
                    const uint8_t* p = row + (x0 + i) * 3;
                    s0 += (int)p[0] * k[i];
                    s1 += (int)p[1] * k[i];
                    s2 += (int)p[2] * k[i];
                }
                m[0] = pp_clip8(s0);
                m[1] = pp_clip8(s1);
                m[2] = pp_clip8(s2);
            } else {
                m[0] = row[x * 3];
                m[1] = row[x * 3 + 1];
                m[2] = row[x * 3 + 2];
            }
        }
        __syncthreads();
        // second pass: vertical -> output rows of the band, 4 consecutive x per thread
        const int ow4 = ow >> 2;
        for (int it = tid; it < nb * ow4; it += 256) {
            const int yi = it / ow4, x = (it % ow4) * 4;
            uint8_t p[4][3];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                if (need_v) {
                    const int y0 = vb[2 * yi] - r0, n = vb[2 * yi + 1];
                    const int* k = vk + yi * KV;
                    int s0 = 1 << (PP_PREC - 1), s1 = s0, s2 = s0;
                    for (int j = 0; j < n; j++) {
                        const uint8_t* q = mid + ((int64_t)(y0 + j) * ow + x + u) * 3;
                        s0 += (int)q[0] * k[j];
                        s1 += (int)q[1] * k[j];
                        s2 += (int)q[2] * k[j];
                    }
                    p[u][0] = pp_clip8(s0);
                    p[u][1] = pp_clip8(s1);
                    p[u][2] = pp_clip8(s2);
                } else {
                    const uint8_t* q = mid + ((int64_t)yi * ow + x + u) * 3;
                    p[u][0] = q[0];
                    p[u][1] = q[1];
                    p[u][2] = q[2];
                }
            }
            emit4(yi, x, 0, p);
            emit4(yi, x, 1, p);
            emit4(yi, x, 2, p);
        }
    } else {
        // tall narrow source (h > 100 w): vertical first over all w columns -> mid[yi][x'][c]
        for (int it = tid; it < nb * w; it += 256) {
            const int yi = it / w, x = it % w;
            const int y0 = vb[2 * yi], n = vb[2 * yi + 1];
            const int* k = vk + yi * KV;
            int s0 = 1 << (PP_PREC - 1), s1 = s0, s2 = s0;
            for (int j = 0; j < n; j++) {
                const uint8_t* p = src + ((int64_t)(y0 + j) * w + x) * 3;
                s0 += (int)p[0] * k[j];
                s1 += (int)p[1] * k[j];
                s2 += (int)p[2] * k[j];
            }
            uint8_t* m = mid + (int64_t)it * 3;
            m[0] = pp_clip8(s0);
            m[1] = pp_clip8(s1);
            m[2] = pp_clip8(s2);
        }
        __syncthreads();
        const int ow4 = ow >> 2;
        for (int it = tid; it < nb * ow4; it += 256) {
            const int yi = it / ow4, x = (it % ow4) * 4;
            uint8_t p[4][3];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int x0 = hb[2 * (x + u)], n = hb[2 * (x + u) + 1];
                const int* k = hk + (x + u) * KH;
                int s0 = 1 << (PP_PREC - 1), s1 = s0, s2 = s0;
                for (int i = 0; i < n; i++) {
                    const uint8_t* q = mid + ((int64_t)yi * w + x0 + i) * 3;
                    s0 += (int)q[0] * k[i];
                    s1 += (int)q[1] * k[i];
                    s2 += (int)q[2] * k[i];
                }
                p[u][0] = pp_clip8(s0);
                p[u][1] = pp_clip8(s1);
                p[u][2] = pp_clip8(s2);
            }
            emit4(yi, x, 0, p);
            emit4(yi, x, 1, p);
            emit4(yi, x, 2, p);
        }
    }
}

// LDS bytes of preprocess_kernel for a batch whose sources are at most max_h x max_w.
static size_t pp_lds_bytes(int oh, int ow, int max_h, int max_w, int* kh_cap, int* kv_cap, int* rows_cap) {
    *kh_cap = pp_ksize(max_w, ow);
    *kv_cap = pp_ksize(max_h, oh);
    // source rows read by one band: span of PP_BAND consecutive filter windows
    // <= (BAND - 1) * scale + 2 * support + 2 (window ends are rounded by at most 1/2 each)
    const double sv = (double)max_h / oh, supp = sv < 1.0 ? 1.0 : sv;
    *rows_cap = (int)((PP_BAND - 1) * sv + 2 * supp + 2) + 2;
    if (*rows_cap < PP_BAND) *rows_cap = PP_BAND;
    const size_t mid_h = (size_t)(*rows_cap) * ow * 3, mid_v = (size_t)PP_BAND * max_w * 3;
    const size_t mid = mid_h > mid_v ? mid_h : mid_v;
    return (768 + 2 * (size_t)ow + (size_t)ow * (*kh_cap) + 2 * PP_BAND + (size_t)PP_BAND * (*kv_cap)) * 4 + mid;
}

}  // namespace reidmi

using namespace reidmi;

REIDMI_API int reidmi_preprocess_lds_size(int oh, int ow, int max_h, int max_w, int64_t* bytes) {
    RM_REQUIRE(oh > 0 && ow > 0 && max_h > 0 && max_w > 0 && bytes, "preprocess: bad sizes");
    int a, b, c;
    *bytes = (int64_t)pp_lds_bytes(oh, ow, max_h, max_w, &a, &b, &c);
    return OK;
}

REIDMI_API int reidmi_preprocess_u8(const uint8_t* pix, const int64_t* meta, int64_t B, int max_h, int max_w, int oh,
                                    int ow, const float* mean, const float* stdv, int out_dtype, void* out,
                                    void* stream) {
    RM_REQUIRE(B >= 0 && oh > 0 && ow > 0 && max_h > 0 && max_w > 0, "preprocess: bad sizes");
    RM_REQUIRE(oh <= 65535 * PP_BAND && B <= 65535, "preprocess: grid too large (split the batch)");
    RM_REQUIRE(out_dtype == 0 || out_dtype == 1, "preprocess: out_dtype must be 0 (fp32) or 1 (fp16)");
    RM_REQUIRE(ow % 4 == 0, "preprocess: output width must be a multiple of 4");
    RM_REQUIRE(mean && stdv && out && (B == 0 || (pix && meta)), "preprocess: null pointer");
    if (B == 0) return OK;
    PPArgs a{};
    a.pix = pix;
    a.meta = meta;
    a.oh = oh;
    a.ow = ow;
    a.max_h = max_h;
    a.max_w = max_w;
    const size_t lds = pp_lds_bytes(oh, ow, max_h, max_w, &a.kh_cap, &a.kv_cap, &a.rows_cap);
    RM_REQUIRE(lds <= 160 * 1024, "preprocess: source images too large for the on-chip band (max_h / oh or "
                                  "max_w / ow too big): resize on the host first");
    for (int c = 0; c < 3; c++) {
        RM_REQUIRE(stdv[c] != 0.0f, "preprocess: std must be non-zero");
        a.mean[c] = mean[c];
        a.stdv[c] = stdv[c];
    }
    a.out_f16 = out_dtype;
    a.out = out;
    static size_t attr = 0;
    if (lds > 64 * 1024 && lds > attr) {
        RM_CHECK_HIP(hipFuncSetAttribute((const void*)preprocess_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                         (int)lds));
        attr = lds;
    }
    hipLaunchKernelGGL(preprocess_kernel, dim3((unsigned)ceil_div(oh, PP_BAND), (unsigned)B), dim3(256), lds,
                       (hipStream_t)stream, a);
    RM_LAUNCHED();
    return OK;
}
