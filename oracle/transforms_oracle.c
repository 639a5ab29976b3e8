/*
 * transforms_oracle.c — CPU restatement of the reference's test-time image transforms.
 *
 * TEST INFRASTRUCTURE ONLY (see reid_oracle.c): the checker for reidmi_preprocess_u8.
 *
 * The reference (data_prepare.py:257-270) builds
 *     transforms.Resize((256, 128)) -> ToTensor() -> Normalize((0.5,)*3, (0.5,)*3)
 * on a PIL RGB image (data_prepare.py:88, Image.open(...).convert("RGB")).  torchvision
 * (absent here) hands a PIL image to PIL.Image.resize((w, h), BILINEAR) (its `antialias`
 * flag only concerns tensors); so the arithmetic lives in the third-party dependency
 * Pillow — version used to pin it here: Pillow 12.2.0 (libImaging/Resample.c).  Its
 * published algorithm, restated:
 *   precompute_coeffs (per axis, in double):
 *     scale = in/out; fs = max(scale, 1); support = 1.0 (bilinear) * fs;
 *     ksize = ceil(support)*2 + 1
 *     for each output x: center = (x + 0.5) * scale; ss = 1/fs
 *       xmin = max((int)(center - support + 0.5), 0); xmax = min((int)(center + support + 0.5), in) - xmin
 *       w_i = tri((i + xmin - center + 0.5) * ss), tri(t) = max(1 - |t|, 0); w_i /= sum(w) (if sum != 0)
 *   normalize_coeffs_8bpc: k_i = (int)(w_i * 2^22 +/- 0.5)   (PRECISION_BITS = 32 - 8 - 2)
 *   two passes, each skipped when that axis keeps its size, horizontal first — except
 *   for tall narrow sources shrunk vertically (h > 100*w and oh < h), where Pillow 12.2
 *   runs the vertical pass first (pass order identified by probing Pillow here: on every
 *   probed (h, w, oh, ow) exactly one order reproduces it, and this rule picks it):
 *     out = clip8((2^21 + sum_i k_i * in[xmin + i]) >> 22),  clip8 = clamp to [0, 255]
 *   (an arithmetic shift: floor).
 *   ToTensor: float32(p) / 255 (correctly rounded); Normalize: (v - 0.5f) / 0.5f.
 * Pinned bit-exact against Pillow itself on random images of many sizes
 * (tests/golden/make_transform_goldens.py -> tests/golden/transforms.npz; tests/test_oracle.py).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORC_PREC 22

static double orc_tri(double x) {
    if (x < 0.0) x = -x;
    if (x < 1.0) return 1.0 - x;
    return 0.0;
}

/* Coefficients of one axis.  bounds[2*o] = first source index, bounds[2*o+1] = count;
 * kk[o*ksize + i] fixed-point weights.  Returns ksize (kk must hold out*ksize ints;
 * pass kk = NULL to query ksize). */
int orc_resize_coeffs(int in_size, int out_size, int32_t* bounds, int32_t* kk) {
    const double scale = (double)((float)in_size - 0.0f) / out_size;
    const double fs = scale < 1.0 ? 1.0 : scale;
    const double support = 1.0 * fs;
    const int ksize = (int)ceil(support) * 2 + 1;
    if (!kk) return ksize;
    double* w = (double*)malloc(sizeof(double) * (size_t)ksize);
    for (int o = 0; o < out_size; o++) {
        const double center = 0.0 + (o + 0.5) * scale;
        const double ss = 1.0 / fs;
        int xmin = (int)(center - support + 0.5);
        if (xmin < 0) xmin = 0;
        int xmax = (int)(center + support + 0.5);
        if (xmax > in_size) xmax = in_size;
        xmax -= xmin;
        double ww = 0.0;
        int i;
        for (i = 0; i < xmax; i++) {
            const double t = orc_tri((i + xmin - center + 0.5) * ss);
            w[i] = t;
            ww += t;
        }
        for (i = 0; i < xmax; i++)
            if (ww != 0.0) w[i] /= ww;
        for (; i < ksize; i++) w[i] = 0.0;
        for (i = 0; i < ksize; i++)
            kk[(size_t)o * ksize + i] = w[i] < 0 ? (int32_t)(-0.5 + w[i] * (1 << ORC_PREC))
                                                 : (int32_t)(0.5 + w[i] * (1 << ORC_PREC));
        bounds[2 * o] = xmin;
        bounds[2 * o + 1] = xmax;
    }
    free(w);
    return ksize;
}

static uint8_t orc_clip8(int32_t v) {
    v >>= ORC_PREC;
    return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
}

/* One separable pass over an HWC uint8 image: resample axis `ax` (0 = rows, 1 = columns)
 * from n_in to n_out with the coefficients of orc_resize_coeffs. */
static void orc_pass(const uint8_t* src, int h, int w, int ax, int n_out, uint8_t* dst) {
    const int n_in = ax == 0 ? h : w;
    const int k = orc_resize_coeffs(n_in, n_out, NULL, NULL);
    int32_t* b = (int32_t*)malloc(sizeof(int32_t) * 2 * (size_t)n_out);
    int32_t* kk = (int32_t*)malloc(sizeof(int32_t) * (size_t)n_out * k);
    orc_resize_coeffs(n_in, n_out, b, kk);
    const int oh = ax == 0 ? n_out : h, ow = ax == 0 ? w : n_out;
    for (int y = 0; y < oh; y++)
        for (int x = 0; x < ow; x++)
            for (int c = 0; c < 3; c++) {
                const int o = ax == 0 ? y : x;
                const int first = b[2 * o], n = b[2 * o + 1];
                int32_t ss = 1 << (ORC_PREC - 1);
                for (int i = 0; i < n; i++) {
                    const int yy = ax == 0 ? first + i : y, xx = ax == 0 ? x : first + i;
                    ss += (int32_t)src[((size_t)yy * w + xx) * 3 + c] * kk[(size_t)o * k + i];
                }
                dst[((size_t)y * ow + x) * 3 + c] = orc_clip8(ss);
            }
    free(b);
    free(kk);
}

/* 1 if Pillow 12.2 runs the vertical pass first for this resize (see header). */
int orc_resize_vertical_first(int h, int w, int oh, int ow) {
    return ow != w && oh != h && oh < h && (int64_t)h > 100 * (int64_t)w;
}

/* PIL.Image.resize((ow, oh), BILINEAR) of an RGB image; src/dst HWC uint8.  (Restricting the
 * first pass to the lines the second one reads, as Pillow does, changes no value.) */
void orc_pil_resize_rgb(const uint8_t* src, int h, int w, int oh, int ow, uint8_t* dst) {
    const int need_h = ow != w, need_v = oh != h;
    if (need_h && need_v) {
        const int vfirst = orc_resize_vertical_first(h, w, oh, ow);
        uint8_t* tmp = (uint8_t*)malloc((size_t)(vfirst ? oh * w : h * ow) * 3);
        if (vfirst) {
            orc_pass(src, h, w, 0, oh, tmp);
            orc_pass(tmp, oh, w, 1, ow, dst);
        } else {
            orc_pass(src, h, w, 1, ow, tmp);
            orc_pass(tmp, h, ow, 0, oh, dst);
        }
        free(tmp);
    } else if (need_h) {
        orc_pass(src, h, w, 1, ow, dst);
    } else if (need_v) {
        orc_pass(src, h, w, 0, oh, dst);
    } else {
        memcpy(dst, src, (size_t)h * w * 3);
    }
}

/* ToTensor + Normalize(mean, std) (per channel): HWC uint8 -> CHW float32. */
void orc_to_tensor_normalize(const uint8_t* hwc, int h, int w, const float* mean, const float* std, float* chw) {
    for (int c = 0; c < 3; c++)
        for (int y = 0; y < h; y++)
            for (int x = 0; x < w; x++) {
                const float v = (float)hwc[((size_t)y * w + x) * 3 + c] / 255.0f;
                chw[((size_t)c * h + y) * w + x] = (v - mean[c]) / std[c];
            }
}
