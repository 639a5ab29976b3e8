// Development check of jpeg_core.h on the host (no GPU needed): runs the same per-image
// entropy decode, IDCT and colour code the kernels run, serially, so the arithmetic can be
// compared with Pillow in this container (tools/jpeg_host_check.py).  Not part of the product
// library; the GPU tests compare the device kernels with Pillow directly.
//   hipcc -O2 -std=c++17 -fPIC -shared -I../multimodal-reid_amd/csrc -I../include \
//         jpeg_host_check.hip -o build/libjpeghost.so
#include <cstring>
#include <vector>

#include "jpeg_core.h"

using namespace reidmi::jpeg;

// always_replay: run every image with libjpeg's input buffering replayed (the kernels take the
// decode-only pass first and replay only when the end of the data decides): both must agree.
static int host_decode(const uint8_t* files, const uint8_t* plan, const int64_t* info, uint8_t* out, int32_t* err,
                       bool always_replay) {
    const JpegPlan* P = (const JpegPlan*)plan;
    const JpegImage* imgs = (const JpegImage*)(plan + P->img_off);
    const JpegHuff* huff = (const JpegHuff*)(plan + P->huff_off);
    const int16_t* quant = (const int16_t*)(plan + P->quant_off);
    std::vector<int16_t> coef((size_t)info[6] + 64, 0);
    std::vector<uint8_t> planes((size_t)P->plane_bytes + 64, 0);
    for (int64_t i = 0; i < P->B; ++i) {
        const JpegImage& im = imgs[i];
        err[i] = im.status;
        if (im.status != J_OK) continue;
        DirectSink sink;
        err[i] = always_replay ? J_REPLAY : entropy_decode<false>(files, im, huff, coef.data(), sink);
        if (err[i] == J_REPLAY) err[i] = entropy_decode<true>(files, im, huff, coef.data(), sink);
        for (int c = 0; c < im.ncomp; ++c) {
            const int64_t pitch = (int64_t)im.bw[c] * 8;
            for (int by = 0; by < im.bh[c]; ++by)
                for (int bx = 0; bx < im.bw[c]; ++bx)
                    idct_islow(coef.data() + im.coef_off + im.comp_coef[c] + ((int64_t)by * im.bw[c] + bx) * 64,
                               quant + (int64_t)im.quant[c] * 64,
                               planes.data() + im.plane_off + im.comp_plane[c] + (int64_t)by * 8 * pitch + bx * 8,
                               pitch);
        }
        for (int y = 0; y < im.h; ++y)
            for (int x = 0; x < im.w; ++x) pixel_rgb(im, planes.data() + im.plane_off, x, y, out + im.out_off + ((int64_t)y * im.w + x) * 3);
    }
    return 0;
}

extern "C" int jpeg_host_decode(const uint8_t* files, const uint8_t* plan, const int64_t* info, uint8_t* out,
                                int32_t* err) {
    return host_decode(files, plan, info, out, err, false);
}

extern "C" int jpeg_host_decode_replay(const uint8_t* files, const uint8_t* plan, const int64_t* info, uint8_t* out,
                                       int32_t* err) {
    return host_decode(files, plan, info, out, err, true);
}
