// jpeg.hip — JPEG decode of the reference's loaders on the GPU:
// reidDataset.__getitem__ opens every crop with `Image.open(path).convert("RGB")`
// (data_prepare.py:87-92) in 4 DataLoader workers (data_prepare.py:275-283).  Here a batch of
// baseline JPEG files is decoded on the device, bit-exact with Pillow / libjpeg-turbo, into the
// packed HWC uint8 layout reidmi_preprocess_u8 (transforms.hip) consumes.
//
// Split (the arithmetic lives in jpeg_core.h):
//   host   reidmi_jpeg_plan    — marker parse of each file's headers (a few hundred bytes):
//                                quantisers, Huffman tables (derived once per distinct table),
//                                geometry, workspace / output offsets -> one plan blob;
//   device jpeg_entropy_kernel — one lane per image: the serial Huffman decode (the only
//                                sequential part of JPEG) into int16 coefficient blocks;
//          jpeg_pixels_kernel  — one workgroup per image: islow IDCT of every block into its
//                                component plane (L2-resident), then fancy upsampling +
//                                YCbCr->RGB per output pixel.
// Supported: baseline / extended-sequential Huffman, 8-bit, one scan, grayscale or three
// components at 4:4:4, 4:2:2 or 4:2:0 (every ReID benchmark's crops).  Anything else gets a
// per-image status and is left to the caller (the Python mirror raises).
#include <algorithm>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "common.h"
#include "jpeg_core.h"

namespace reidmi {
namespace jpeg {

// ------------------------------------------------------------------ host: header parse

static void build_huff(const uint8_t* counts, const uint8_t* syms, int nsym, JpegHuff& t) {
    // jdhuff.c jpeg_make_d_derived_tbl: canonical codes by length, then the lookahead table
    memset(&t, 0, sizeof(t));
    int p = 0;
    uint32_t code = 0;
    for (int l = 1; l <= 16; ++l) {
        const int n = counts[l - 1];
        t.valoff[l] = p - (int32_t)code;
        for (int i = 0; i < n; ++i, ++p, ++code) {
            if (l <= kLookahead) {
                const int shift = kLookahead - l;
                for (int e = 0; e < (1 << shift) && (code << shift | e) < (1u << kLookahead); ++e)
                    t.lut[(code << shift) | e] = (uint16_t)((l << 8) | syms[p]);
            }
        }
        t.lim[l] = code << (16 - l);
        code <<= 1;
    }
    t.lim[17] = 0xFFFFFFFFu;
    for (int i = 0; i < nsym && i < 256; ++i) t.val[i] = syms[i];
}

// jdhuff.c jpeg_make_d_derived_tbl's checks on a table the scan uses: no length may hold more
// codes than it has room for (JERR_BAD_HUFF_TABLE), and a DC table's symbols are sizes <= 15
static bool huff_ok(const uint8_t* counts, const uint8_t* syms, int nsym, bool dc) {
    uint32_t code = 0;   // one past the last code of length l: the all-ones code is not allowed
    for (int l = 1; l <= 16; ++l) {
        code += counts[l - 1];
        if (code >= (1u << l)) return false;
        code <<= 1;
    }
    if (dc)
        for (int i = 0; i < nsym; ++i)
            if (syms[i] > 15) return false;
    return true;
}

struct Pools {
    std::vector<JpegHuff> huff;
    std::vector<std::string> huff_raw;   // 16 counts + symbols of each pooled table
    std::vector<int16_t> quant;          // [n][64]

    // Tables repeat across a dataset (one encoder setting: 4 Huffman + 2 quantisation tables),
    // so the lookup is a scan of the few pooled ones, newest first.
    int add_huff(const uint8_t* raw, int len) {
        for (int i = (int)huff_raw.size() - 1; i >= 0; --i)
            if ((int)huff_raw[i].size() == len && memcmp(huff_raw[i].data(), raw, len) == 0) return i;
        JpegHuff t;
        build_huff(raw, raw + 16, len - 16, t);
        huff.push_back(t);
        huff_raw.emplace_back((const char*)raw, len);
        return (int)huff.size() - 1;
    }
    int add_quant(const int16_t* q) {
        for (int i = (int)(quant.size() / 64) - 1; i >= 0; --i)
            if (memcmp(quant.data() + 64 * i, q, 128) == 0) return i;
        quant.insert(quant.end(), q, q + 64);
        return (int)(quant.size() / 64) - 1;
    }
};

static inline int u16be(const uint8_t* p) { return (p[0] << 8) | p[1]; }

// The standard Huffman tables of ITU T.81 Annex K.3 (16 code counts, then the symbols): what
// libjpeg-turbo's jpeg_make_d_derived_tbl substitutes (jstdhuff.c jpeg_std_huff_table) when a
// scan names table 0 or 1 that no DHT defined (Motion-JPEG frames omit them).
static const uint8_t kStdDcLuma[28] = {
    0x00, 0x01, 0x05, 0x01, 0x01, 0x01, 0x01, 0x01, 0x01, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00,
    0x00, 0x01, 0x02, 0x03, 0x04, 0x05, 0x06, 0x07, 0x08, 0x09, 0x0a, 0x0b,
};
static const uint8_t kStdAcLuma[178] = {
    0x00, 0x02, 0x01, 0x03, 0x03, 0x02, 0x04, 0x03, 0x05, 0x05, 0x04, 0x04, 0x00, 0x00, 0x01, 0x7d,
    0x01, 0x02, 0x03, 0x00, 0x04, 0x11, 0x05, 0x12, 0x21, 0x31, 0x41, 0x06, 0x13, 0x51, 0x61, 0x07,
    0x22, 0x71, 0x14, 0x32, 0x81, 0x91, 0xa1, 0x08, 0x23, 0x42, 0xb1, 0xc1, 0x15, 0x52, 0xd1, 0xf0,
    0x24, 0x33, 0x62, 0x72, 0x82, 0x09, 0x0a, 0x16, 0x17, 0x18, 0x19, 0x1a, 0x25, 0x26, 0x27, 0x28,
    0x29, 0x2a, 0x34, 0x35, 0x36, 0x37, 0x38, 0x39, 0x3a, 0x43, 0x44, 0x45, 0x46, 0x47, 0x48, 0x49,
    0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58, 0x59, 0x5a, 0x63, 0x64, 0x65, 0x66, 0x67, 0x68, 0x69,
    0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a, 0x83, 0x84, 0x85, 0x86, 0x87, 0x88, 0x89,
    0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97, 0x98, 0x99, 0x9a, 0xa2, 0xa3, 0xa4, 0xa5, 0xa6, 0xa7,
    0xa8, 0xa9, 0xaa, 0xb2, 0xb3, 0xb4, 0xb5, 0xb6, 0xb7, 0xb8, 0xb9, 0xba, 0xc2, 0xc3, 0xc4, 0xc5,
    0xc6, 0xc7, 0xc8, 0xc9, 0xca, 0xd2, 0xd3, 0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda, 0xe1, 0xe2,
    0xe3, 0xe4, 0xe5, 0xe6, 0xe7, 0xe8, 0xe9, 0xea, 0xf1, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8,
    0xf9, 0xfa,
};
static const uint8_t kStdDcChroma[28] = {
    0x00, 0x03, 0x01, 0x01, 0x01, 0x01, 0x01, 0x01, 0x01, 0x01, 0x01, 0x00, 0x00, 0x00, 0x00, 0x00,
    0x00, 0x01, 0x02, 0x03, 0x04, 0x05, 0x06, 0x07, 0x08, 0x09, 0x0a, 0x0b,
};
static const uint8_t kStdAcChroma[178] = {
    0x00, 0x02, 0x01, 0x02, 0x04, 0x04, 0x03, 0x04, 0x07, 0x05, 0x04, 0x04, 0x00, 0x01, 0x02, 0x77,
    0x00, 0x01, 0x02, 0x03, 0x11, 0x04, 0x05, 0x21, 0x31, 0x06, 0x12, 0x41, 0x51, 0x07, 0x61, 0x71,
    0x13, 0x22, 0x32, 0x81, 0x08, 0x14, 0x42, 0x91, 0xa1, 0xb1, 0xc1, 0x09, 0x23, 0x33, 0x52, 0xf0,
    0x15, 0x62, 0x72, 0xd1, 0x0a, 0x16, 0x24, 0x34, 0xe1, 0x25, 0xf1, 0x17, 0x18, 0x19, 0x1a, 0x26,
    0x27, 0x28, 0x29, 0x2a, 0x35, 0x36, 0x37, 0x38, 0x39, 0x3a, 0x43, 0x44, 0x45, 0x46, 0x47, 0x48,
    0x49, 0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58, 0x59, 0x5a, 0x63, 0x64, 0x65, 0x66, 0x67, 0x68,
    0x69, 0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a, 0x82, 0x83, 0x84, 0x85, 0x86, 0x87,
    0x88, 0x89, 0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97, 0x98, 0x99, 0x9a, 0xa2, 0xa3, 0xa4, 0xa5,
    0xa6, 0xa7, 0xa8, 0xa9, 0xaa, 0xb2, 0xb3, 0xb4, 0xb5, 0xb6, 0xb7, 0xb8, 0xb9, 0xba, 0xc2, 0xc3,
    0xc4, 0xc5, 0xc6, 0xc7, 0xc8, 0xc9, 0xca, 0xd2, 0xd3, 0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda,
    0xe2, 0xe3, 0xe4, 0xe5, 0xe6, 0xe7, 0xe8, 0xe9, 0xea, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8,
    0xf9, 0xfa,
};

// jdmarker.c read_markers up to the first SOS, restricted to what the device decodes.
static int32_t parse_one(const uint8_t* f, int64_t n, int64_t base, JpegImage& im, Pools& pools) {
    memset(&im, 0, sizeof(im));   // (status is set by the caller from the return value)
    // Pillow's JpegImagePlugin accepts only files starting FF D8 FF (_accept)
    if (n < 4 || f[0] != 0xFF || f[1] != 0xD8 || f[2] != 0xFF) return J_NOT_JPEG;
    int64_t p = 2;
    bool jfif = false, adobe = false, sof = false;
    int adobe_t = -1;
    bool qdef[4] = {false, false, false, false};
    int16_t qt[4][64];
    const uint8_t* hdc[4] = {nullptr, nullptr, nullptr, nullptr};
    const uint8_t* hac[4] = {nullptr, nullptr, nullptr, nullptr};
    int hdc_len[4] = {0, 0, 0, 0}, hac_len[4] = {0, 0, 0, 0};
    int cid[3] = {0, 0, 0}, tq[3] = {0, 0, 0};
    for (;;) {
        while (p < n && f[p] != 0xFF) ++p;   // extraneous bytes (libjpeg warns and skips)
        while (p < n && f[p] == 0xFF) ++p;   // fill bytes
        if (p >= n) return J_NOT_JPEG;
        const int m = f[p++];
        if (m == 0x00) continue;   // 0xFF 0x00: skipped like garbage (next_marker)
        // markers outside Pillow's table (TEM, 0x02-0xBF): JpegImagePlugin "no marker found"
        if (m < 0xC0) return J_NOT_JPEG;
        if (m >= 0xD0 && m <= 0xD7) continue;   // RSTn: no parameters
        if (m == 0xD8) return J_NOT_JPEG;   // a second SOI (get_soi: JERR_SOI_DUPLICATE)
        if (m == 0xD9) return J_NOT_JPEG;   // EOI before any scan
        // DHP, EXP, JPGn: skipped by Pillow's parser, then libjpeg's JERR_UNKNOWN_MARKER
        if (m == 0xDE || m == 0xDF || (m >= 0xF0 && m <= 0xFD)) return J_NOT_JPEG;
        if (p + 2 > n) return J_NOT_JPEG;
        const int len = u16be(f + p);
        if (len < 2 || p + len > n) return J_NOT_JPEG;
        const uint8_t* s = f + p + 2;
        const int sl = len - 2;
        if (m == 0xC0 || m == 0xC1) {   // SOF0 baseline / SOF1 extended sequential, Huffman
            if (sl < 6 || s[0] != 8) return J_UNSUPPORTED;
            im.h = u16be(s + 1);
            im.w = u16be(s + 3);
            im.ncomp = s[5];
            if (im.h == 0 || im.w == 0) return J_UNSUPPORTED;   // DNL-defined height
            if (im.ncomp != 1 && im.ncomp != 3) return J_LAYOUT;
            if (len != 8 + 3 * im.ncomp) return J_NOT_JPEG;   // get_sof: JERR_BAD_LENGTH
            for (int c = 0; c < im.ncomp; ++c) {
                cid[c] = s[6 + 3 * c];
                im.hs[c] = s[7 + 3 * c] >> 4;
                im.vs[c] = s[7 + 3 * c] & 15;
                tq[c] = s[8 + 3 * c];
                if (tq[c] > 3) return J_BAD_TABLE;   // jdinput.c latch_quant_tables: JERR_NO_QUANT_TABLE
            }
            for (int c = 0; c < im.ncomp; ++c) im.cid[c] = cid[c];
            sof = true;
        } else if ((m >= 0xC2 && m <= 0xCF) && m != 0xC4 && m != 0xC8 && m != 0xCC) {
            return J_UNSUPPORTED;   // progressive, lossless, hierarchical, arithmetic
        } else if (m == 0xC4) {     // DHT (get_dht: tables while > 16 bytes remain, then exactly none)
            int i = 0;
            while (sl - i > 16) {
                const int tc = (s[i] >> 4) & 1, th = s[i] & 0xEF;   // (bit 4: AC; any other bit: a bad index)
                int tot = 0;
                for (int l = 0; l < 16; ++l) tot += s[i + 1 + l];
                if (th > 3 || tot > 256 || i + 17 + tot > sl) return J_BAD_TABLE;
                (tc ? hac : hdc)[th] = s + i + 1;
                (tc ? hac_len : hdc_len)[th] = 16 + tot;
                i += 17 + tot;
            }
            if (i != sl) return J_BAD_TABLE;   // JERR_BAD_LENGTH
        } else if (m == 0xDB) {     // DQT (get_dqt: any nonzero precision nibble means 16-bit entries)
            int i = 0;
            while (i < sl) {
                const int pq = (s[i] >> 4) ? 1 : 0, t = s[i] & 15;
                if (t > 3 || i + 1 + 64 * (pq + 1) > sl) return J_BAD_TABLE;
                for (int k = 0; k < 64; ++k) {   // kept in zig-zag order; libjpeg's quantval is
                    const int q = pq ? u16be(s + i + 1 + 2 * k) : s[i + 1 + k];   // read as-is
                    // 16-bit entries above int16 (libjpeg keeps UINT16): not decoded here
                    if (q > 32767) return J_UNSUPPORTED;
                    qt[t][k] = (int16_t)q;
                }
                qdef[t] = true;
                i += 1 + 64 * (pq + 1);
            }
        } else if (m == 0xDD) {     // DRI
            if (len != 4) return J_NOT_JPEG;   // get_dri: JERR_BAD_LENGTH
            im.ri = u16be(s);
        } else if (m == 0xE0) {     // examine_app0: a JFIF marker needs APP0_DATA_LEN (14) bytes
            if (sl >= 14 && memcmp(s, "JFIF\0", 5) == 0) jfif = true;
        } else if (m == 0xEE) {
            if (sl >= 12 && memcmp(s, "Adobe", 5) == 0) {
                adobe = true;
                adobe_t = s[11];
            }
        } else if (m == 0xCC) {     // DAC (get_dac: index < 32, DC bounds L <= U, exact length)
            if (sl % 2) return J_NOT_JPEG;
            for (int i = 0; i < sl; i += 2)
                if (s[i] >= 32 || (s[i] < 16 && (s[i + 1] & 15) > (s[i + 1] >> 4))) return J_NOT_JPEG;
        } else if (m == 0xDA) {     // SOS
            if (!sof) return J_NOT_JPEG;
            const int ns = sl > 0 ? s[0] : 0;
            if (len != 2 * ns + 6) return J_NOT_JPEG;   // get_sos: JERR_BAD_LENGTH
            if (ns != im.ncomp || sl < 4 + 2 * ns) return J_UNSUPPORTED;   // one interleaved scan only
            for (int j = 0; j < ns; ++j) {
                if (s[1 + 2 * j] != cid[j]) return J_UNSUPPORTED;   // scan order = frame order
                const int td = s[2 + 2 * j] >> 4, ta = s[2 + 2 * j] & 15;
                if (td > 3 || ta > 3) return J_BAD_TABLE;
                if (!hdc[td] && td < 2) {   // jpeg_std_huff_table
                    hdc[td] = td ? kStdDcChroma : kStdDcLuma;
                    hdc_len[td] = td ? (int)sizeof(kStdDcChroma) : (int)sizeof(kStdDcLuma);
                }
                if (!hac[ta] && ta < 2) {
                    hac[ta] = ta ? kStdAcChroma : kStdAcLuma;
                    hac_len[ta] = ta ? (int)sizeof(kStdAcChroma) : (int)sizeof(kStdAcLuma);
                }
                if (!hdc[td] || !hac[ta]) return J_BAD_TABLE;
                if (!huff_ok(hdc[td], hdc[td] + 16, hdc_len[td] - 16, true) ||
                    !huff_ok(hac[ta], hac[ta] + 16, hac_len[ta] - 16, false))
                    return J_BAD_TABLE;
                im.dc[j] = pools.add_huff(hdc[td], hdc_len[td]);
                im.ac[j] = pools.add_huff(hac[ta], hac_len[ta]);
            }
            // Ss, Se, Ah/Al of a sequential scan are only checked by a warning (jdhuff.c
            // start_pass_huff_decoder: JWRN_NOT_SEQUENTIAL) and then ignored
            im.src_off = base + p + len;
            im.src_len = n - (p + len);
            break;
        }
        p += len;
    }
    for (int c = 0; c < im.ncomp; ++c) {
        if (!qdef[tq[c]]) return J_BAD_TABLE;
        im.quant[c] = pools.add_quant(qt[tq[c]]);
    }
    // geometry (jdinput.c initial_setup, per_scan_setup)
    if (im.ncomp == 1) {
        im.hs[0] = im.vs[0] = 1;
        im.mcux = (im.w + 7) / 8;
        im.mcuy = (im.h + 7) / 8;
        im.bw[0] = im.mcux;
        im.bh[0] = im.mcuy;
        im.dw[0] = im.w;
        im.dh[0] = im.h;
        im.cspace = CS_GRAY;
    } else {
        const int h0 = im.hs[0], v0 = im.vs[0];
        for (int c = 1; c < 3; ++c)
            if (im.hs[c] != 1 || im.vs[c] != 1) return J_LAYOUT;
        if (!((h0 == 1 && v0 == 1) || (h0 == 2 && v0 == 1) || (h0 == 2 && v0 == 2))) return J_LAYOUT;
        im.mcux = (im.w + 8 * h0 - 1) / (8 * h0);
        im.mcuy = (im.h + 8 * v0 - 1) / (8 * v0);
        for (int c = 0; c < 3; ++c) {
            im.bw[c] = im.mcux * im.hs[c];
            im.bh[c] = im.mcuy * im.vs[c];
            im.dw[c] = (int)(((int64_t)im.w * im.hs[c] + h0 - 1) / h0);
            im.dh[c] = (int)(((int64_t)im.h * im.vs[c] + v0 - 1) / v0);
        }
        // jdapimin.c default_decompress_parms (3 components)
        if (jfif) im.cspace = CS_YCC;
        else if (adobe) im.cspace = adobe_t == 0 ? CS_RGB : CS_YCC;
        else if (cid[0] == 82 && cid[1] == 71 && cid[2] == 66) im.cspace = CS_RGB;
        else im.cspace = CS_YCC;
    }
    if ((int64_t)im.w * im.h > (int64_t)1 << 26) return J_UNSUPPORTED;   // > 64 Mpixel
    return J_OK;
}

static inline int64_t align_up(int64_t v, int64_t a) { return (v + a - 1) / a * a; }

// ------------------------------------------------------------------ device

constexpr int kLdsTables = 8;   // Huffman tables staged in LDS per workgroup (4 per encoder setting)

// kLds: the plan's table pool (n_huff <= kLdsTables, the usual case) is copied to LDS and every
// lookup is a ds_read (a generic pointer would compile to flat loads, whose waits also drain
// the lane's outstanding global loads and stores).
// Each lane assembles its current block in LDS (ds_write per coefficient) and stores it whole
// (8 x 16 bytes) when the block ends, so no global store sits between a refill's word load
// and its use, and the coefficient workspace needs no clearing.
struct LdsSink {
    int16_t* buf;   // this lane's 64 slots in LDS
    int16_t* dst;
    __device__ inline void begin(int16_t* b) {
        dst = b;
        uint4* q = (uint4*)buf;
#pragma unroll
        for (int j = 0; j < 8; ++j) q[j] = make_uint4(0, 0, 0, 0);
    }
    __device__ inline void put(int k, int32_t v) { buf[k] = (int16_t)v; }
    __device__ inline void end() {
        const uint4* q = (const uint4*)buf;
        uint4* d = (uint4*)dst;
#pragma unroll
        for (int j = 0; j < 8; ++j) d[j] = q[j];
    }
};

// kLds: the plan's table pool (n_huff <= kLdsTables, the usual case) is copied to LDS and every
// lookup is a ds_read (a generic pointer would compile to flat loads, whose waits also drain
// the lane's outstanding global loads and stores).
template <bool kLds>
__global__ __launch_bounds__(64) void jpeg_entropy_kernel(const uint8_t* __restrict__ src,
                                                          const uint8_t* __restrict__ plan, int64_t B,
                                                          int16_t* __restrict__ coef, int32_t* __restrict__ err) {
    __shared__ JpegHuff lds[kLds ? kLdsTables : 1];
    __shared__ __attribute__((aligned(16))) int16_t blocks[64][64];
    const JpegPlan* P = (const JpegPlan*)plan;
    const JpegHuff* gh = (const JpegHuff*)(plan + P->huff_off);
    if constexpr (kLds) {
        const uint4* g = (const uint4*)gh;
        uint4* l = (uint4*)lds;
        const int64_t nh = P->n_huff < kLdsTables ? P->n_huff : kLdsTables;   // (the host checked n_huff)
        const int n16 = (int)(nh * (int64_t)sizeof(JpegHuff) / 16);
        for (int j = threadIdx.x; j < n16; j += 64) l[j] = g[j];
        __syncthreads();
    }
    const int64_t i = (int64_t)blockIdx.x * 64 + threadIdx.x;
    if (i >= B) return;
    const JpegImage im = ((const JpegImage*)(plan + P->img_off))[i];
    int32_t st = im.status;
    if (st == J_OK) {
        LdsSink sink{blocks[threadIdx.x], nullptr};
        // the decode alone first; libjpeg's input buffering is replayed beside a second decode
        // only for the images whose end of data decides (no marker after the scan, or restart
        // intervals): a lane that needs it runs while the others of its wave wait
        if constexpr (kLds) st = entropy_decode<false>(src, im, lds, coef, sink);
        else st = entropy_decode<false>(src, im, gh, coef, sink);
        if (st == J_REPLAY) {
            if constexpr (kLds) st = entropy_decode<true>(src, im, lds, coef, sink);
            else st = entropy_decode<true>(src, im, gh, coef, sink);
        }
        // undecodable data: the image's coefficients are defined as zero (a truncated file keeps
        // what libjpeg would decode, the missing data as zeros: check=False callers get that image)
        if (st != J_OK && st != J_TRUNCATED) {
            int64_t n = 0;
            for (int c = 0; c < im.ncomp; ++c) n += (int64_t)im.bw[c] * im.bh[c] * 64;
            uint4* d = (uint4*)(coef + im.coef_off);
            for (int64_t j = 0; j < n / 8; ++j) d[j] = make_uint4(0, 0, 0, 0);
        }
    }
    err[i] = st;
}

constexpr int64_t kPlaneLds = 64 << 10;   // images whose planes fit stage them in LDS

// kLds: the image's component planes live in (dynamic) LDS between the IDCT and the colour
// pass; otherwise in the plane workspace (L2-resident at these sizes).
template <bool kLds>
__global__ __launch_bounds__(256) void jpeg_pixels_kernel(const uint8_t* __restrict__ plan,
                                                          const int16_t* __restrict__ coef,
                                                          uint8_t* __restrict__ planes, uint8_t* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) uint8_t jpeg_planes_lds[];
    const JpegPlan* P = (const JpegPlan*)plan;
    const JpegImage im = ((const JpegImage*)(plan + P->img_off))[blockIdx.x];
    if (im.status != J_OK) return;
    uint8_t* ip = kLds ? jpeg_planes_lds : planes + im.plane_off;
    const int16_t* qbase = (const int16_t*)(plan + P->quant_off);
    const int nc = im.ncomp;
    const int64_t n0 = (int64_t)im.bw[0] * im.bh[0];
    const int64_t n1 = nc > 1 ? (int64_t)im.bw[1] * im.bh[1] : 0;
    const int64_t nblk = n0 + (nc > 1 ? 2 * n1 : 0);
    for (int64_t t = threadIdx.x; t < nblk; t += 256) {
        int c;
        int64_t local;
        if (t < n0) {
            c = 0;
            local = t;
        } else {
            c = t < n0 + n1 ? 1 : 2;
            local = t - n0 - (c == 2 ? n1 : 0);
        }
        const int bw = c == 0 ? im.bw[0] : (c == 1 ? im.bw[1] : im.bw[2]);
        const int64_t by = local / bw, bx = local - by * bw;
        const int64_t pitch = (int64_t)bw * 8;
        const int qi = c == 0 ? im.quant[0] : (c == 1 ? im.quant[1] : im.quant[2]);
        const int64_t cc = c == 0 ? im.comp_coef[0] : (c == 1 ? im.comp_coef[1] : im.comp_coef[2]);
        const int64_t cp = c == 0 ? im.comp_plane[0] : (c == 1 ? im.comp_plane[1] : im.comp_plane[2]);
        idct_islow(coef + im.coef_off + cc + local * 64, qbase + (int64_t)qi * 64, ip + cp + by * 8 * pitch + bx * 8,
                   pitch);
    }
    __syncthreads();
    // pixels in raster order, 256 apart per thread: (x, y) advances by (256 mod w, 256 / w)
    // without a division per pixel
    const int w = im.w;
    const int sy = 256 / w, sx = 256 - sy * w;
    int y = (int)threadIdx.x / w;
    int x = (int)threadIdx.x - y * w;
    uint8_t* o = out + im.out_off;
    while (y < im.h) {
        uint8_t rgb[3];
        pixel_rgb(im, ip, x, y, rgb);
        uint8_t* d = o + ((int64_t)y * w + x) * 3;
        d[0] = rgb[0];
        d[1] = rgb[1];
        d[2] = rgb[2];
        x += sx;
        y += sy;
        if (x >= w) {
            x -= w;
            ++y;
        }
    }
}

}  // namespace jpeg
}  // namespace reidmi

using namespace reidmi;
using namespace reidmi::jpeg;

REIDMI_API int reidmi_jpeg_plan(const uint8_t* files, const int64_t* offsets, int64_t B, void* plan,
                                int64_t plan_capacity, int64_t* meta, int32_t* status, int64_t* info) {
    RM_REQUIRE(B >= 0 && info != nullptr && (B == 0 || (files && offsets && meta && status)),
               "reidmi_jpeg_plan: bad arguments");
    for (int64_t i = 0; i < B; ++i)
        RM_REQUIRE(offsets[i] >= 0 && offsets[i + 1] >= offsets[i], "reidmi_jpeg_plan: offsets must be non-decreasing from 0");
    std::vector<JpegImage> imgs((size_t)B);
    // headers parse independently: chunks on host threads, each with its own table pool, merged after
    const int nt = (int)std::max<int64_t>(1, std::min<int64_t>({16, (int64_t)std::thread::hardware_concurrency(),
                                                               B / 2048}));
    std::vector<Pools> local((size_t)nt);
    auto work = [&](int t) {
        for (int64_t i = B * t / nt; i < B * (t + 1) / nt; ++i) {
            const int64_t a = offsets[i];
            imgs[(size_t)i].status = parse_one(files + a, offsets[i + 1] - a, a, imgs[(size_t)i], local[(size_t)t]);
        }
    };
    if (nt == 1) {
        work(0);
    } else {
        std::vector<std::thread> th;
        for (int t = 0; t < nt; ++t) th.emplace_back(work, t);
        for (auto& x : th) x.join();
    }
    Pools pools;
    std::vector<std::vector<int>> hmap((size_t)nt), qmap((size_t)nt);
    for (int t = 0; t < nt; ++t) {
        const Pools& L = local[(size_t)t];
        for (size_t j = 0; j < L.huff_raw.size(); ++j)
            hmap[(size_t)t].push_back(pools.add_huff((const uint8_t*)L.huff_raw[j].data(), (int)L.huff_raw[j].size()));
        for (size_t j = 0; j < L.quant.size() / 64; ++j) qmap[(size_t)t].push_back(pools.add_quant(L.quant.data() + 64 * j));
    }
    int64_t coef = 0, plane = 0, outb = 0, max_h = 0, max_w = 0, bad = 0, max_plane = 0;
    for (int64_t i = 0; i < B; ++i) {
        JpegImage& im = imgs[(size_t)i];
        const int32_t st = im.status;
        status[i] = st;
        if (st != J_OK) {
            meta[3 * i] = meta[3 * i + 1] = meta[3 * i + 2] = 0;
            ++bad;
            continue;
        }
        int t = 0;
        while (t + 1 < nt && i >= B * (t + 1) / nt) ++t;
        for (int c = 0; c < im.ncomp; ++c) {
            im.dc[c] = hmap[(size_t)t][(size_t)im.dc[c]];
            im.ac[c] = hmap[(size_t)t][(size_t)im.ac[c]];
            im.quant[c] = qmap[(size_t)t][(size_t)im.quant[c]];
        }
        im.coef_off = coef;
        im.plane_off = plane;
        int64_t cc = 0;
        for (int c = 0; c < im.ncomp; ++c) {
            im.comp_coef[c] = cc;
            im.comp_plane[c] = cc;   // one byte per coefficient slot: the same relative layout
            cc += (int64_t)im.bw[c] * im.bh[c] * 64;
        }
        coef += cc;
        plane += cc;
        max_plane = cc > max_plane ? cc : max_plane;
        im.out_off = outb;
        meta[3 * i] = outb;
        meta[3 * i + 1] = im.h;
        meta[3 * i + 2] = im.w;
        outb += (int64_t)im.w * im.h * 3;
        max_h = im.h > max_h ? im.h : max_h;
        max_w = im.w > max_w ? im.w : max_w;
    }
    JpegPlan hdr;
    hdr.B = B;
    hdr.n_huff = (int64_t)pools.huff.size();
    hdr.n_quant = (int64_t)pools.quant.size() / 64;
    hdr.img_off = align_up(sizeof(JpegPlan), 64);
    hdr.huff_off = align_up(hdr.img_off + B * (int64_t)sizeof(JpegImage), 64);
    hdr.quant_off = align_up(hdr.huff_off + hdr.n_huff * (int64_t)sizeof(JpegHuff), 64);
    hdr.coef_elems = coef;
    hdr.plane_bytes = plane;
    hdr.out_bytes = outb;
    const int64_t plan_bytes = hdr.quant_off + hdr.n_quant * 128;
    info[0] = plan_bytes;
    info[1] = align_up(coef * 2, 256) + plane;   // workspace: int16 coefficients, then planes
    info[2] = outb;
    info[3] = max_h;
    info[4] = max_w;
    info[5] = bad;
    info[6] = coef;
    info[7] = hdr.n_huff;
    info[8] = max_plane;
    info[9] = B;
    if (plan == nullptr || plan_capacity < plan_bytes) return OK;   // sizing call
    uint8_t* pb = (uint8_t*)plan;
    memset(pb, 0, (size_t)plan_bytes);
    memcpy(pb, &hdr, sizeof(hdr));
    if (B) memcpy(pb + hdr.img_off, imgs.data(), (size_t)B * sizeof(JpegImage));
    if (hdr.n_huff) memcpy(pb + hdr.huff_off, pools.huff.data(), pools.huff.size() * sizeof(JpegHuff));
    if (hdr.n_quant) memcpy(pb + hdr.quant_off, pools.quant.data(), pools.quant.size() * sizeof(int16_t));
    return OK;
}

REIDMI_API int reidmi_jpeg_decode(const uint8_t* files, const void* plan, const int64_t* info, int64_t B, void* ws,
                                  int64_t ws_bytes, uint8_t* pix, int32_t* err, void* stream) {
    RM_REQUIRE(info != nullptr && B >= 0, "reidmi_jpeg_decode: bad arguments");
    if (B == 0) return OK;
    RM_REQUIRE(files && plan && ws && err && (pix || info[2] == 0), "reidmi_jpeg_decode: null pointer");
    RM_REQUIRE(ws_bytes >= info[1], "reidmi_jpeg_decode: workspace smaller than info[1]");
    RM_REQUIRE(info[9] == B, "reidmi_jpeg_decode: B differs from the plan's (info[9])");
    hipStream_t s = (hipStream_t)stream;
    int16_t* coef = (int16_t*)ws;
    uint8_t* planes = (uint8_t*)ws + align_up(info[6] * 2, 256);
    const dim3 eg((unsigned)((B + 63) / 64));
    if (info[7] <= kLdsTables)
        jpeg_entropy_kernel<true><<<eg, dim3(64), 0, s>>>(files, (const uint8_t*)plan, B, coef, err);
    else
        jpeg_entropy_kernel<false><<<eg, dim3(64), 0, s>>>(files, (const uint8_t*)plan, B, coef, err);
    RM_LAUNCHED();
    if (info[8] <= kPlaneLds)
        jpeg_pixels_kernel<true><<<dim3((unsigned)B), dim3(256), (size_t)info[8], s>>>((const uint8_t*)plan, coef,
                                                                                       planes, pix);
    else
        jpeg_pixels_kernel<false><<<dim3((unsigned)B), dim3(256), 0, s>>>((const uint8_t*)plan, coef, planes, pix);
    RM_LAUNCHED();
    return OK;
}

// ------------------------------------------------------------------ host: the loader's file reads
// reidDataset.__getitem__ opens one file per item in 4 DataLoader worker processes
// (data_prepare.py:87-89, 275-283); here one batch of files lands in one caller-owned pinned
// buffer (the H2D copy source of the decode) from up to 16 host threads, each taking a
// contiguous range of items holding ~1/nt of the bytes.

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

namespace {

int loader_threads(int nthreads, int64_t n, int64_t bytes) {
    const int64_t hw = std::max<int64_t>(1, (int64_t)std::thread::hardware_concurrency());
    int64_t nt = nthreads > 0 ? nthreads : std::min<int64_t>(16, hw);
    nt = std::min<int64_t>({nt, std::max<int64_t>(1, n), std::max<int64_t>(1, bytes >> 20)});   // >= 1 MiB each
    return (int)std::max<int64_t>(1, nt);
}

// items [first[t], first[t + 1]) for thread t: equal shares of the bytes (offsets is the prefix sum)
template <class F>
void over_items(const int64_t* offsets, int64_t n, int nt, F&& f) {
    if (nt <= 1 || n <= 1) {
        f((int64_t)0, n);
        return;
    }
    std::vector<int64_t> first((size_t)nt + 1, n);
    first[0] = 0;
    const int64_t total = offsets[n] - offsets[0];
    for (int t = 1; t < nt; ++t) {
        const int64_t target = offsets[0] + total * t / nt;
        first[(size_t)t] = std::lower_bound(offsets, offsets + n, target) - offsets;
        first[(size_t)t] = std::max(first[(size_t)t], first[(size_t)t - 1]);
    }
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t) th.emplace_back([&, t] { f(first[(size_t)t], first[(size_t)t + 1]); });
    for (auto& x : th) x.join();
}

}  // namespace

REIDMI_API int reidmi_files_size(const char* const* paths, int64_t n, int64_t* sizes, int nthreads) {
    RM_REQUIRE(n >= 0 && (n == 0 || (paths && sizes)), "reidmi_files_size: bad arguments");
    std::vector<int64_t> idx((size_t)n + 1);
    for (int64_t i = 0; i <= n; ++i) idx[(size_t)i] = i;   // equal item counts per thread
    over_items(idx.data(), n, loader_threads(nthreads, n, n << 20), [&](int64_t a, int64_t b) {
        for (int64_t i = a; i < b; ++i) {
            struct stat sb;
            sizes[i] = (paths[i] != nullptr && stat(paths[i], &sb) == 0 && S_ISREG(sb.st_mode)) ? (int64_t)sb.st_size : -1;
        }
    });
    return OK;
}

REIDMI_API int reidmi_files_read(const char* const* paths, int64_t n, const int64_t* offsets, uint8_t* dst,
                                 int32_t* status, int nthreads) {
    RM_REQUIRE(n >= 0 && (n == 0 || (paths && offsets && status && (dst || offsets[n] == offsets[0]))),
               "reidmi_files_read: bad arguments");
    for (int64_t i = 0; i < n; ++i)
        RM_REQUIRE(offsets[i + 1] >= offsets[i] && offsets[i] >= 0, "reidmi_files_read: offsets must be non-decreasing from >= 0");
    over_items(offsets, n, loader_threads(nthreads, n, offsets[n] - offsets[0]), [&](int64_t a, int64_t b) {
        for (int64_t i = a; i < b; ++i) {
            const int64_t want = offsets[i + 1] - offsets[i];
            const int fd = paths[i] ? open(paths[i], O_RDONLY | O_CLOEXEC) : -1;
            if (fd < 0) {
                status[i] = 1;
                continue;
            }
            int64_t got = 0;
            int32_t st = 0;
            while (got < want) {
                const ssize_t r = pread(fd, dst + offsets[i] + got, (size_t)(want - got), (off_t)got);
                if (r < 0) {
                    st = 1;
                    break;
                }
                if (r == 0) break;
                got += r;
            }
            if (st == 0 && got != want) st = 2;
            if (st == 0) {   // a longer file than its stated size is a size mismatch too
                uint8_t extra;
                if (pread(fd, &extra, 1, (off_t)want) == 1) st = 2;
            }
            close(fd);
            status[i] = st;
        }
    });
    return OK;
}

REIDMI_API int reidmi_bytes_gather(const void* const* srcs, int64_t n, const int64_t* offsets, uint8_t* dst,
                                   int nthreads) {
    RM_REQUIRE(n >= 0 && (n == 0 || (srcs && offsets && (dst || offsets[n] == offsets[0]))),
               "reidmi_bytes_gather: bad arguments");
    for (int64_t i = 0; i < n; ++i) {
        RM_REQUIRE(offsets[i + 1] >= offsets[i] && offsets[i] >= 0, "reidmi_bytes_gather: offsets must be non-decreasing from >= 0");
        RM_REQUIRE(srcs[i] != nullptr || offsets[i + 1] == offsets[i], "reidmi_bytes_gather: null source");
    }
    over_items(offsets, n, loader_threads(nthreads, n, offsets[n] - offsets[0]), [&](int64_t a, int64_t b) {
        for (int64_t i = a; i < b; ++i)
            if (offsets[i + 1] > offsets[i]) memcpy(dst + offsets[i], srcs[i], (size_t)(offsets[i + 1] - offsets[i]));
    });
    return OK;
}
