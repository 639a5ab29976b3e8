// jpeg_core.h — baseline-JPEG decode arithmetic shared by the device kernels (jpeg.hip) and
// the host-side check tool (tools/jpeg_host_check.hip).  What it reproduces, bit for bit, is
// the decoder behind the reference's `Image.open(path).convert("RGB")` (data_prepare.py:89):
// Pillow 12.2 on libjpeg-turbo (jpeg 6.2 API) with its defaults — Huffman sequential decode,
// the "islow" integer IDCT (LL&M, 13-bit constants, 2 extra bits between passes), "fancy"
// triangular chroma upsampling for 2x1 and 2x2 subsampling, and the 16-bit fixed-point
// YCbCr -> RGB tables.  The published algorithm is restated here; the GPU tests pin it
// against Pillow's own output.
//
// A decode plan (built on the host by reidmi_jpeg_plan from the file headers) is one
// position-independent blob: JpegPlan | JpegImage[B] | JpegHuff[n_huff] | int16 quant[n_quant][64]
// (quantisers, like the coefficients, in zig-zag order).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace reidmi {
namespace jpeg {

// per-image status (reidmi_jpeg_plan / reidmi_jpeg_decode)
enum : int32_t {
    J_OK = 0,
    J_NOT_JPEG = 1,        // no SOI / truncated headers
    J_UNSUPPORTED = 2,     // progressive, lossless, arithmetic-coded, 12-bit, multi-scan
    J_LAYOUT = 3,          // component count / sampling factors outside 1, 3 x {4:4:4, 4:2:2, 4:2:0}
    J_BAD_TABLE = 4,       // missing or malformed DQT / DHT
    J_BAD_DATA = 5,        // entropy-coded data does not decode (set by the device pass)
    J_TRUNCATED = 6,       // libjpeg's input starves before the last MCU (Pillow: "image file is truncated")
    J_REPLAY = 100,        // internal: decode again with libjpeg's input buffering replayed (LjInput)
};

enum : int32_t { CS_GRAY = 0, CS_YCC = 1, CS_RGB = 2 };

struct JpegHuff {          // jdhuff.c-style derived table
    uint16_t lut[1 << 10]; // 10-bit lookahead: (code length << 8) | symbol, 0 = longer code
    uint32_t lim[18];      // left-justified 16-bit bound of all codes of length <= l
    int32_t valoff[18];    // symbol index of a length-l code = code + valoff[l]
    uint8_t val[256];
};

static_assert(sizeof(JpegHuff) % 16 == 0, "JpegHuff is staged to LDS in 16-byte words");

struct JpegImage {
    int64_t src_off, src_len;   // entropy-coded data (after SOS) in the file batch
    int64_t coef_off;           // int16 elements into the coefficient workspace
    int64_t plane_off;          // bytes into the plane workspace
    int64_t out_off;            // bytes into the RGB output (HWC uint8)
    int64_t comp_coef[3];       // per component, relative to coef_off
    int64_t comp_plane[3];      // per component, relative to plane_off
    int32_t w, h, ncomp, cspace;
    int32_t mcux, mcuy, ri, status;   // MCUs per row / column, restart interval (MCUs)
    int32_t hs[3], vs[3];       // sampling factors (1 or 2)
    int32_t bw[3], bh[3];       // blocks per row / column (whole MCUs)
    int32_t dw[3], dh[3];       // downsampled component size (libjpeg downsampled_width/height)
    int32_t quant[3], dc[3], ac[3];   // pool indices
    int32_t cid[3];             // frame component identifiers (the post-scan SOS checks)
};

struct JpegPlan {
    int64_t B, n_huff, n_quant;
    int64_t img_off, huff_off, quant_off;   // bytes from the plan start
    int64_t coef_elems, plane_bytes, out_bytes;
};

// natural (row-major) index -> zig-zag position.  Coefficients and quantisers are kept in
// zig-zag (stream) order; the IDCT's fully unrolled loads apply this permutation at compile time.
constexpr uint8_t kZz[64] = {0,  1,  5,  6,  14, 15, 27, 28, 2,  4,  7,  13, 16, 26, 29, 42,
                             3,  8,  12, 17, 25, 30, 41, 43, 9,  11, 18, 24, 31, 40, 44, 53,
                             10, 19, 23, 32, 39, 45, 52, 54, 20, 22, 33, 38, 46, 51, 55, 60,
                             21, 34, 37, 47, 50, 56, 59, 61, 35, 36, 48, 49, 57, 58, 62, 63};

// ---------------------------------------------------------------- entropy decode (one image)
// jdhuff.c decode_mcu for a single interleaved (or single-component) baseline scan, written as
// one flat loop over Huffman symbols so that the lanes of a wave (one image each) stay
// converged: one iteration = one DC or AC symbol.  Bits are read MSB first from a 64-bit
// window; 0xFF00 is a stuffed 0xFF; any other marker stops the stream (zeros are fed, as
// libjpeg does) until the restart logic skips an RSTn.
constexpr int kLookahead = 10;

struct BitReader {
    const uint8_t* p;
    const uint8_t* end;
    uint64_t acc;   // MSB-aligned bit window
    int bits;       // valid bits in acc
    bool marker;    // a marker (or the end) was reached: zeros are fed from here on
    int64_t loaded; // bits moved into acc since start() (fillers after a marker included):
                    // the bits consumed in the segment are loaded - bits
    int64_t real;   // the segment's data bits (loaded when the marker was reached)
    bool nw_ok;     // nw0/nw1: the aligned words covering >= 5 stream bytes at p, loaded one
    int nmis;       // refill ahead and first read at the next refill, so the load's latency
    uint32_t nw0, nw1;   // hides behind the symbols decoded in between

    __host__ __device__ inline void fetch() {
        nw_ok = !marker && p + 8 <= end;
        if (nw_ok) {
            nmis = (int)((uintptr_t)p & 3);
            const uint32_t* w = (const uint32_t*)(p - nmis);   // (pointer arithmetic keeps it a global load)
            nw0 = w[0];
            nw1 = w[1];
        }
    }
    __host__ __device__ inline void start(const uint8_t* b, const uint8_t* e) {
        p = b;
        end = e;
        acc = 0;
        bits = 0;
        loaded = 0;
        real = INT64_MAX;
        marker = false;
        fetch();
    }
    // a decode step used bits past the segment's data (jdhuff.c jpeg_fill_bit_buffer: the
    // request exceeds what precedes the marker -> insufficient_data)
    __host__ __device__ inline bool past_data() const { return loaded - bits > real; }
    // Keeps >= 32 bits in the window (a symbol plus its extra bits is at most 17 + 15).  The
    // next 4 stream bytes come from the prefetched words: all four at once when none is 0xFF,
    // else one at a time in registers (0xFF 0x00 is a stuffed 0xFF, 0xFF + anything but 0x00 /
    // 0xFF a marker) — no memory access either way.  0xFF 0xFF (fill bytes, which libjpeg reads
    // up to the byte after them: 0x00 makes them one 0xFF data byte, anything else a marker) and
    // the last 8 bytes of a stream go byte by byte.
    __host__ __device__ inline void refill() {
        if (bits >= 32) return;
        bool bytewise = !nw_ok;
        if (nw_ok) {
            const uint64_t win = (((uint64_t)nw1 << 32) | nw0) >> (nmis * 8);   // stream bytes, LSB first
            const uint32_t x = ~(uint32_t)win;
            if (((x - 0x01010101u) & ~x & 0x80808080u) == 0) {
                const uint32_t v = (uint32_t)win;
                const uint32_t be = (v >> 24) | ((v >> 8) & 0xFF00u) | ((v << 8) & 0xFF0000u) | (v << 24);
                acc |= (uint64_t)be << (32 - bits);
                bits += 32;
                loaded += 32;
                p += 4;
            } else {
                int pos = 0;
                while (pos < 4 && bits < 32) {
                    const uint32_t c = (uint32_t)(win >> (8 * pos)) & 0xFF;
                    if (c == 0xFF) {
                        const uint32_t n = (uint32_t)(win >> (8 * pos + 8)) & 0xFF;
                        if (n == 0xFF) {   // fill bytes: the byte loop below reads past them
                            bytewise = true;
                            break;
                        }
                        if (n != 0) {
                            marker = true;
                            real = loaded;
                            break;
                        }
                        pos += 2;
                    } else {
                        pos += 1;
                    }
                    acc |= (uint64_t)c << (56 - bits);
                    bits += 8;
                    loaded += 8;
                }
                p += pos;
                if (marker && bits < 32) {   // zeros from here on
                    loaded += 32 - bits;
                    bits = 32;
                }
                // each stuffed pair takes two window bytes for 8 bits: from a short window
                // (e.g. 5 bits + FF 00 FF 00 = 21) the byte loop tops it up to >= 32
                if (!marker && bits < 32) bytewise = true;
            }
            if (!bytewise) {
                fetch();
                return;
            }
        }
        while (bits < 32) {
            uint32_t c = 0;
            if (!marker) {
                if (p >= end) {
                    marker = true;
                    real = loaded;
                } else {
                    c = p[0];
                    if (c == 0xFF) {
                        const uint8_t* q = p + 1;
                        while (q < end && *q == 0xFF) ++q;
                        if (q < end && *q == 0) {
                            p = q + 1;   // (0xFF)+ 0x00: one 0xFF data byte
                        } else {
                            marker = true;   // p stays at the first 0xFF
                            real = loaded;
                            c = 0;
                        }
                    } else {
                        ++p;
                    }
                }
            }
            acc |= (uint64_t)c << (56 - bits);
            bits += 8;
            loaded += 8;
        }
        fetch();
    }
    __host__ __device__ inline int64_t consumed() const { return loaded - bits; }
    __host__ __device__ inline uint32_t take(int n) {   // n in [1, 16]
        const uint32_t v = (uint32_t)(acc >> (64 - n));
        acc <<= n;
        bits -= n;
        return v;
    }
    // jpeg_huff_decode: returns the symbol.  Codes longer than the lookahead: the length is
    // K+1 + #{l in K+1..16 : lim[l] <= code} (lim is monotone), evaluated without a loop so that
    // the lanes of a wave do not diverge on it.  A code matching no table entry is libjpeg's
    // JWRN_HUFF_BAD_CODE warning: 17 bits consumed, symbol 0 (decoding goes on).
    __host__ __device__ inline int decode(const JpegHuff* t) {
        const uint32_t e = t->lut[acc >> (64 - kLookahead)];
        if (e >> 8) {
            const int l = (int)(e >> 8);
            acc <<= l;
            bits -= l;
            return (int)(e & 0xFF);
        }
        const uint32_t code16 = (uint32_t)(acc >> 48);
        int l = kLookahead + 1;
#pragma unroll
        for (int j = kLookahead + 1; j <= 16; ++j) l += code16 >= t->lim[j] ? 1 : 0;
        if (l > 16) {
            acc <<= 17;
            bits -= 17;
            return 0;
        }
        const int32_t c = (int32_t)(code16 >> (16 - l));
        acc <<= l;
        bits -= l;
        return t->val[(c + t->valoff[l]) & 0xFF];
    }
};

__host__ __device__ inline int32_t huff_extend(uint32_t v, int s) {   // HUFF_EXTEND
    return (v < (1u << (s - 1))) ? (int32_t)v - (1 << s) + 1 : (int32_t)v;
}

// libjpeg-turbo's entropy-decoder input buffering (jdhuff.c), replayed beside the decode to tell
// whether the reference's loader gets the whole image.  Pillow hands libjpeg the file's bytes as
// a suspending source (JpegDecode.c): when a fetch of the bit buffer reaches the end of the data
// before a marker, libjpeg suspends, and at the end of the file Pillow raises "image file is
// truncated"; once every MCU is decoded, a missing EOI does not matter (JpegDecode.c ignores
// jpeg_finish_decompress suspending when all rows are out).  So a file is truncated exactly when
// a fetch during the MCUs (or the search for a restart marker) starves.  Fetch points:
//  * slow path (decode_mcu_slow; every MCU when a restart interval is set, and every MCU that
//    starts with fewer than 512 x blocks_in_MCU bytes left in the buffer): before a Huffman
//    symbol when fewer than 8 bits are buffered, before a symbol's extra bits (or the rest of a
//    code longer than 8 bits) when fewer than those are buffered; a fetch reads bytes until >= 25
//    bits are buffered (MIN_GET_BITS), stopping at a marker (no suspension; zeros follow);
//  * fast path (decode_mcu_fast): 6 bytes whenever <= 16 bits are buffered, before each symbol
//    and each symbol's extra bits; never near the end of the data (the 512-byte margin).
// F counts destuffed bytes fetched in the restart segment, C the bits consumed (BitReader).
#ifndef LJ_MIN_GET_BITS
#define LJ_MIN_GET_BITS 57
#endif
constexpr int kLjMinGetBits = LJ_MIN_GET_BITS;   // BIT_BUF_SIZE - 7 with a 64-bit bit buffer
struct LjInput {
    const uint8_t* p;   // libjpeg's next raw byte
    const uint8_t* end;
    int64_t F;
    bool marker;        // reached a marker (cinfo->unread_marker; p stays at its 0xFF): no more fetches
    bool starved;       // a fetch reached the end of the data first (the loader raises)
    bool fast;          // the current MCU runs decode_mcu_fast
    int next_rst;       // cinfo->marker->next_restart_num
    __host__ __device__ inline void start(const uint8_t* b, const uint8_t* e) {
        p = b;
        end = e;
        F = 0;
        marker = false;
    }
    __host__ __device__ inline void fetch1() {   // one destuffed byte (jpeg_fill_bit_buffer)
        if (p >= end) {
            starved = marker = true;
            return;
        }
        if (*p != 0xFF) {
            ++p;
            ++F;
            return;
        }
        const uint8_t* q = p + 1;
        while (q < end && *q == 0xFF) ++q;   // fill bytes
        if (q >= end) {
            starved = marker = true;
            return;
        }
        if (*q == 0) {
            p = q + 1;
            ++F;
        } else {
            marker = true;   // unread_marker: the bytes stay for the marker reader
        }
    }
    // before reading n bits (n >= 1) at consumed position C
    __host__ __device__ inline void need(int64_t C, int n) {
        if (fast) {
            if (8 * F - C <= 16)   // FILL_BIT_BUFFER_FAST: six FILL_BYTEs (no end check: the margin)
                for (int i = 0; i < 6 && !marker; ++i) fetch1();
        } else if (!marker && 8 * F - C < n) {
            while (!marker && 8 * F - C < kLjMinGetBits) fetch1();
        }
    }
    // a Huffman code of l > 8 bits read from C (jpeg_huff_decode: CHECK_BIT_BUFFER(9), then one
    // bit at a time: a fetch where the buffer ran dry)
    __host__ __device__ inline void need_long(int64_t C, int l) {
        if (fast || marker) return;   // (the fast path's buffer holds > 16 bits here)
        if (8 * F - C < 9) {
            need(C, 9);
        } else if (8 * F - C < l) {
            const int64_t Cd = 8 * F;
            while (!marker && 8 * F - Cd < kLjMinGetBits) fetch1();
        }
    }
    // at an MCU start: decode_mcu's choice of path
    __host__ __device__ inline void mcu(int blocks_in_mcu, bool restarts) {
        fast = !restarts && !marker && (end - p) >= 512 * (int64_t)blocks_in_mcu;
    }
    // jdmarker.c next_marker from q: garbage, 0xFF fill and 0xFF 0x00 skipped; the marker's first
    // 0xFF at *at, its code m, the input after it at *after.  False: the data ends first.
    __host__ __device__ static inline bool next_marker(const uint8_t* q, const uint8_t* e, const uint8_t** at, int* m,
                                                       const uint8_t** after) {
        for (;;) {
            while (q < e && *q != 0xFF) ++q;
            const uint8_t* r = q + 1;
            while (r < e && *r == 0xFF) ++r;
            if (r >= e) return false;
            if (*r != 0) {
                *at = q;
                *m = *r;
                *after = r + 1;
                return true;
            }
            q = r + 1;
        }
    }
    // jdhuff.c process_restart -> jdmarker.c read_restart_marker (+ jpeg_resync_to_restart): the
    // marker a fetch stopped at (or the next one) is the expected RSTn and is consumed, or the
    // resync decides: discard it and resume (1), scan on to the next marker (2), or leave it
    // unread (3: the entropy decoder then reads zeros — an empty segment).  Starves at the end.
    // Returns whether a marker is left unread.
    __host__ __device__ inline bool restart() {
        const uint8_t *at, *after;
        int m;
        if (!next_marker(p, end, &at, &m, &after)) {
            starved = true;
            start(end, end);
            return false;
        }
        bool unread = false;
        for (;;) {
            const int d = next_rst;
            int action;
            if (m == 0xD0 + d) action = 1;                                                    // the expected RSTn
            else if (m < 0xC0) action = 2;                                                    // invalid marker
            else if (m < 0xD0 || m > 0xD7) action = 3;                                        // a non-restart marker
            else if (m == 0xD0 + ((d + 1) & 7) || m == 0xD0 + ((d + 2) & 7)) action = 3;     // one of the next two
            else if (m == 0xD0 + ((d + 7) & 7) || m == 0xD0 + ((d + 6) & 7)) action = 2;     // a prior one
            else action = 1;
            if (action == 1) {
                start(after, end);
                break;
            }
            if (action == 3) {
                start(at, end);
                marker = true;
                unread = true;
                break;
            }
            if (!next_marker(after, end, &at, &m, &after)) {
                starved = true;
                start(end, end);
                return false;
            }
        }
        next_rst = (next_rst + 1) & 7;
        return unread;
    }
};

// Where decoded coefficients go.  DirectSink writes them into zeroed blocks in place (host
// check); the device kernel stages each block in LDS and writes it out whole (jpeg.hip).
struct DirectSink {
    int16_t* blk;
    __host__ __device__ inline void begin(int16_t* b) { blk = b; }
    __host__ __device__ inline void put(int k, int32_t v) { blk[k] = (int16_t)v; }
    __host__ __device__ inline void end() {}
};

// After the scan: libjpeg's jpeg_finish_decompress reads markers until EOI (jdmarker.c
// read_markers / next_marker; a single-scan image).  Suspension (the data ends, anywhere) is fine
// once every row is out (Pillow's JpegDecode.c); an error is the loader raising ("broken data
// stream").  From q: garbage bytes, 0xFF fill and 0xFF00 are skipped to the next marker; EOI ends
// the image; SOI, any SOFn, JPG and the reserved markers are errors; RSTn / TEM take no
// parameters; SOS is an error once its header is read (JERR_EOI_EXPECTED), or earlier when its
// length or a component selector is invalid (get_sos, libjpeg-turbo's two component checks);
// DQT / DHT / DAC / DRI are parsed with get_dqt / get_dht / get_dac / get_dri's checks
// (a DQT table is read whole whatever the length says); APPn / COM / DNL are skipped by length.
// Checked against Pillow 12.2 on fuzzed marker sequences (tests/test_jpeg.py tail_cases).
__host__ __device__ inline int32_t post_scan_status(const uint8_t* q, const uint8_t* end, const JpegImage& im) {
    for (;;) {
        while (q + 1 < end && !(q[0] == 0xFF && q[1] != 0xFF && q[1] != 0)) ++q;
        if (q + 1 >= end) return J_OK;
        const int m = q[1];
        q += 2;
        if (m == 0xD9) return J_OK;
        if (m == 0xD8 || (m >= 0xC0 && m <= 0xCF && m != 0xC4 && m != 0xCC)) return J_BAD_DATA;
        if ((m >= 0xD0 && m <= 0xD7) || m == 0x01) continue;
        if (m == 0xDA) {
            if (end - q < 3) return J_OK;
            const int len = (q[0] << 8) | q[1], ns = q[2];
            if (len != ns * 2 + 6 || ns < 1 || ns > 4) return J_BAD_DATA;
            const uint8_t* r = q + 3;
            int cur[4] = {-1, -1, -1, -1};   // cinfo->cur_comp_info[i]: the component of selector i
            const int nc = im.ncomp < 4 ? im.ncomp : 4;
            for (int i = 0; i < ns; ++i) {
                if (end - r < 2) return J_OK;
                const int cc = r[0];
                r += 2;
                int found = -1;
                for (int ci = 0; ci < nc && found < 0; ++ci)   // (tested at index ci, stored at i)
                    if (im.cid[ci] == cc && cur[ci] < 0) found = ci;
                if (found < 0) return J_BAD_DATA;
                cur[i] = found;
                for (int pi = 0; pi < i; ++pi)
                    if (cur[pi] == found) return J_BAD_DATA;
            }
            return end - r < 3 ? J_OK : J_BAD_DATA;
        }
        const bool seg = m == 0xDD || m == 0xDB || m == 0xC4 || m == 0xCC || m == 0xFE || m == 0xDC ||
                         (m >= 0xE0 && m <= 0xEF);
        if (!seg) return J_BAD_DATA;   // DHP, EXP, JPGn, reserved: JERR_UNKNOWN_MARKER
        if (end - q < 2) return J_OK;
        const int len = (q[0] << 8) | q[1];
        const uint8_t* r = q + 2;
        int64_t length = len - 2;
        if (m == 0xDD) {
            if (len != 4) return J_BAD_DATA;
            if (end - r < 2) return J_OK;
            q = r + 2;
        } else if (m == 0xDB) {
            while (length > 0) {
                --length;
                if (r >= end) return J_OK;
                const int t = *r++;
                if ((t & 15) >= 4) return J_BAD_DATA;
                const int need = (t >> 4) ? 128 : 64;
                if (end - r < need) return J_OK;
                r += need;
                length -= need;
            }
            if (length != 0) return J_BAD_DATA;
            q = r;
        } else if (m == 0xC4) {
            while (length > 16) {
                if (end - r < 17) return J_OK;
                int idx = r[0], count = 0;
                for (int l = 1; l <= 16; ++l) count += r[l];
                r += 17;
                length -= 17;
                if (count > 256 || count > length) return J_BAD_DATA;
                if (end - r < count) return J_OK;
                r += count;
                length -= count;
                if (idx & 0x10) idx -= 0x10;
                if (idx >= 4) return J_BAD_DATA;
            }
            if (length != 0) return J_BAD_DATA;
            q = r;
        } else if (m == 0xCC) {
            while (length > 0) {
                if (end - r < 2) return J_OK;
                const int idx = r[0], val = r[1];
                r += 2;
                length -= 2;
                if (idx >= 32) return J_BAD_DATA;
                if (idx < 16 && (val & 15) > (val >> 4)) return J_BAD_DATA;
            }
            if (length != 0) return J_BAD_DATA;
            q = r;
        } else {   // APPn, COM, DNL: skip_variable / get_interesting_appn
            q = r + (length > 0 ? length : 0);
        }
    }
}

// Decodes one image's scan into zig-zag-order int16 coefficient blocks.  Returns J_OK,
// J_BAD_DATA (then the blocks not yet ended are left as they were) or J_TRUNCATED (libjpeg's
// input would starve before the last MCU, LjInput: every block is decoded, missing data as zeros,
// but the reference's loader raises for such a file).  kReplay = false runs the decode alone and
// returns J_REPLAY when the end of the data decides (no marker after the scan, or restart
// intervals, whose marker search the replay follows): the caller decodes again with kReplay.
template <bool kReplay, class Sink>
__host__ __device__ inline int32_t entropy_decode(const uint8_t* src, const JpegImage& im, const JpegHuff* huff,
                                                  int16_t* coef, Sink& sink) {
    // One iteration = one symbol, with the DC and AC cases folded into the same arithmetic
    // (DC: run 0, size = symbol, value added to the component's predictor) and the block
    // position kept as running per-component MCU origins, so that lanes at different points
    // of their streams execute nearly the same instructions.
    if constexpr (!kReplay)
        if (im.ri) return J_REPLAY;
    BitReader br;
    br.start(src + im.src_off, src + im.src_off + im.src_len);
    LjInput lj;
    lj.starved = false;
    lj.next_rst = 0;
    lj.start(src + im.src_off, src + im.src_off + im.src_len);
    const bool gray = im.ncomp == 1;
    const int h0 = gray ? 1 : im.hs[0];
    const int n0 = gray ? 1 : im.hs[0] * im.vs[0];   // Y blocks per MCU
    const int nb = gray ? 1 : n0 + 2;                // blocks per MCU
    const int64_t nmcu = (int64_t)im.mcux * im.mcuy;
    const JpegHuff* dct0 = huff + im.dc[0];
    const JpegHuff* dct1 = huff + im.dc[gray ? 0 : 1];
    const JpegHuff* dct2 = huff + im.dc[gray ? 0 : 2];
    const JpegHuff* act0 = huff + im.ac[0];
    const JpegHuff* act1 = huff + im.ac[gray ? 0 : 1];
    const JpegHuff* act2 = huff + im.ac[gray ? 0 : 2];
    const int64_t bw0 = im.bw[0];
    int16_t* org0 = coef + im.coef_off + im.comp_coef[0];   // MCU origins per component
    int16_t* org1 = coef + im.coef_off + im.comp_coef[1];
    int16_t* org2 = coef + im.coef_off + im.comp_coef[2];
    const int64_t row_skip0 = gray ? 0 : (int64_t)(im.vs[0] - 1) * bw0 * 64;   // Y rows of an MCU beyond the first
    int32_t pred0 = 0, pred1 = 0, pred2 = 0;
    int64_t mcu = 0;
    int mx = 0, b = 0, k = 0;
    int togo = im.ri;   // MCUs left in this restart interval
    int comp = 0;
    sink.begin(org0);
    const JpegHuff* tbl = dct0;
    if constexpr (kReplay) lj.mcu(nb, im.ri != 0);
    // jdhuff.c decode_mcu: once a step of the segment used bits past its data (a marker, or
    // the end, reached too early), the MCU finishes on zero bits and the segment's later MCUs
    // are left zero (insufficient_data, cleared at a restart): one loop iteration per block then
    bool skip = false;
    while (mcu < nmcu) {
        if (skip) {
            k = 64;
        } else {
            br.refill();
            const int64_t c0 = br.consumed();
            if constexpr (kReplay) lj.need(c0, 8);   // HUFF_DECODE (HUFF_DECODE_FAST)
            const int sym = br.decode(tbl);
            const int64_t c1 = br.consumed();
            if constexpr (kReplay)
                if (c1 - c0 > 8) lj.need_long(c0, (int)(c1 - c0));   // a code longer than the lookahead
            const bool dc = k == 0;
            const int r = dc ? 0 : sym >> 4;
            const int s = dc ? sym : sym & 15;
            if (s > 15) return J_BAD_DATA;
            if constexpr (kReplay)
                if (s) lj.need(c1, s);   // CHECK_BIT_BUFFER(s) / FILL_BIT_BUFFER_FAST
            int32_t v = s ? huff_extend(br.take(s), s) : 0;
            if (dc) {
                v += comp == 0 ? pred0 : (comp == 1 ? pred1 : pred2);
                pred0 = comp == 0 ? v : pred0;
                pred1 = comp == 1 ? v : pred1;
                pred2 = comp == 2 ? v : pred2;
                tbl = comp == 0 ? act0 : (comp == 1 ? act1 : act2);
            }
            k += r;
            if (s || dc) {
                // a run past the block: libjpeg's jpeg_natural_order[] extra entries map k 64..79
                // to position 63 (damaged data)
                sink.put(k > 63 ? 63 : k, v);
                k += 1;
            } else {
                k = r == 15 ? k + 1 : 64;   // ZRL: 16 zeros; EOB
            }
        }
        if (k >= 64) {   // block done: the next block of the MCU, or the next MCU
            sink.end();
            k = 0;
            if (++b == nb) {
                b = 0;
                ++mcu;
                skip = skip || br.past_data();
                org0 += h0 * 64;
                org1 += 64;
                org2 += 64;
                if (++mx == im.mcux) {
                    mx = 0;
                    org0 += row_skip0;
                }
                if (im.ri && mcu < nmcu && --togo == 0) {
                    togo = im.ri;
                    pred0 = pred1 = pred2 = 0;
                    if constexpr (kReplay) {   // (restart intervals always take the replay)
                        // libjpeg discards the buffered bits and continues where its input is;
                        // a marker left unread feeds zeros (insufficient_data is kept then)
                        const bool unread = lj.restart();
                        br.start(lj.p, lj.end);
                        if (unread) {
                            br.marker = true;
                            br.real = 0;
                            br.nw_ok = false;
                        } else {
                            skip = false;
                        }
                    }
                }
                if constexpr (kReplay) lj.mcu(nb, im.ri != 0);
            }
            comp = b < n0 ? 0 : b - n0 + 1;
            int16_t* y = org0 + ((b & (h0 - 1)) + (int64_t)(b >> (h0 - 1)) * bw0) * 64;
            sink.begin(comp == 0 ? y : (comp == 1 ? org1 : org2));
            tbl = comp == 0 ? dct0 : (comp == 1 ? dct1 : dct2);
        }
    }
    // every MCU decoded: the reference's loader returns the image unless libjpeg's input starved
    // on the way (LjInput); a missing EOI alone does not fail it.  Without the replay, the scan is
    // known not to starve when a marker follows the data: with no restart interval libjpeg's
    // fetches never pass the first marker after the scan start, and the BitReader stops at or
    // before it, so a marker found from br.p is one libjpeg's input never reached past.
    // Otherwise (no marker before the end) the decode runs again with the replay.
    const uint8_t* q;
    if constexpr (kReplay) {
        if (lj.starved) return J_TRUNCATED;
        q = lj.p;
    } else {
        q = br.p;
        while (q + 1 < br.end && !(q[0] == 0xFF && q[1] != 0xFF && q[1] != 0)) ++q;
        if (q + 1 >= br.end) return J_REPLAY;
    }
    return post_scan_status(q, br.end, im);
}

// ---------------------------------------------------------------- islow IDCT (jidctint.c)
constexpr int CB = 13, P1 = 2;   // CONST_BITS, PASS1_BITS
constexpr int32_t F0298 = 2446, F0390 = 3196, F0541 = 4433, F0765 = 6270, F0899 = 7373, F1175 = 9633,
                  F1501 = 12299, F1847 = 15137, F1961 = 16069, F2053 = 16819, F2562 = 20995, F3072 = 25172;

template <typename T>
__host__ __device__ inline T descale(T x, int n) { return (x + ((T)1 << (n - 1))) >> n; }

// IDCT_range_limit[x & RANGE_MASK] of jdmaster.c prepare_range_limit_table (8-bit samples)
__host__ __device__ inline uint8_t idct_limit(int32_t x) {
    const int32_t v = x & 1023;
    if (v < 128) return (uint8_t)(v + 128);
    if (v < 512) return 255;
    if (v < 896) return 0;
    return (uint8_t)(v - 896);
}

// one 1-D 8-point pass of the LL&M butterfly on d[0..7] (stride st), dequantised inputs.
// libjpeg-turbo computes it in JLONG (64-bit); T = int32_t is the same arithmetic whenever no
// intermediate leaves int32, which idct_islow checks per block (kPass1Max / kPass2Max).
template <typename T>
struct Idct8 {
    T t10, t11, t12, t13, o0, o1, o2, o3;
    __host__ __device__ inline void run(T d0, T d1, T d2, T d3, T d4, T d5, T d6, T d7) {
        T z1 = (d2 + d6) * F0541;
        const T tmp2 = z1 + d6 * (-F1847);
        const T tmp3 = z1 + d2 * F0765;
        const T tmp0 = (d0 + d4) * ((T)1 << CB);
        const T tmp1 = (d0 - d4) * ((T)1 << CB);
        t10 = tmp0 + tmp3;
        t13 = tmp0 - tmp3;
        t11 = tmp1 + tmp2;
        t12 = tmp1 - tmp2;
        T a0 = d7, a1 = d5, a2 = d3, a3 = d1;
        z1 = a0 + a3;
        T z2 = a1 + a2, z3 = a0 + a2, z4 = a1 + a3;
        const T z5 = (z3 + z4) * F1175;
        a0 *= F0298;
        a1 *= F2053;
        a2 *= F3072;
        a3 *= F1501;
        z1 *= -F0899;
        z2 *= -F2562;
        z3 *= -F1961;
        z4 *= -F0390;
        z3 += z5;
        z4 += z5;
        o0 = a0 + z1 + z3;
        o1 = a1 + z2 + z4;
        o2 = a2 + z2 + z3;
        o3 = a3 + z1 + z4;
    }
};

// Every intermediate of one Idct8 pass is at most 178 219 x max|input| in magnitude (the sum of
// the absolute butterfly constants along the longest path), so with max|input| <= these bounds
// the int32 pass equals libjpeg's 64-bit one.  Valid images stay far below them; damaged entropy
// data (huge coefficients) takes the 64-bit pass, as libjpeg computes it.
constexpr int32_t kPass1Max = 12000;   // 178 219 x 12 000 < 2^31
constexpr int32_t kPass2Max = 12000;

template <typename T>
__host__ __device__ inline void idct_pass1(const int32_t (&dq)[64], int32_t (&ws)[64]) {
#pragma unroll
    for (int c = 0; c < 8; ++c) {   // pass 1: columns
        Idct8<T> t;
        t.run(dq[0 * 8 + c], dq[1 * 8 + c], dq[2 * 8 + c], dq[3 * 8 + c], dq[4 * 8 + c], dq[5 * 8 + c], dq[6 * 8 + c],
              dq[7 * 8 + c]);
        // (int) DESCALE(...): libjpeg stores the workspace as int (a 64-bit value truncates)
        ws[0 * 8 + c] = (int32_t)descale<T>(t.t10 + t.o3, CB - P1);
        ws[7 * 8 + c] = (int32_t)descale<T>(t.t10 - t.o3, CB - P1);
        ws[1 * 8 + c] = (int32_t)descale<T>(t.t11 + t.o2, CB - P1);
        ws[6 * 8 + c] = (int32_t)descale<T>(t.t11 - t.o2, CB - P1);
        ws[2 * 8 + c] = (int32_t)descale<T>(t.t12 + t.o1, CB - P1);
        ws[5 * 8 + c] = (int32_t)descale<T>(t.t12 - t.o1, CB - P1);
        ws[3 * 8 + c] = (int32_t)descale<T>(t.t13 + t.o0, CB - P1);
        ws[4 * 8 + c] = (int32_t)descale<T>(t.t13 - t.o0, CB - P1);
    }
}

template <typename T>
__host__ __device__ inline uint64_t idct_row(const int32_t* w) {
    Idct8<T> t;
    t.run(w[0], w[1], w[2], w[3], w[4], w[5], w[6], w[7]);
    constexpr int S = CB + P1 + 3;
    // (int) DESCALE(...) & RANGE_MASK: the low 10 bits survive the truncation
    const uint32_t o0 = idct_limit((int32_t)descale<T>(t.t10 + t.o3, S));
    const uint32_t o7 = idct_limit((int32_t)descale<T>(t.t10 - t.o3, S));
    const uint32_t o1 = idct_limit((int32_t)descale<T>(t.t11 + t.o2, S));
    const uint32_t o6 = idct_limit((int32_t)descale<T>(t.t11 - t.o2, S));
    const uint32_t o2 = idct_limit((int32_t)descale<T>(t.t12 + t.o1, S));
    const uint32_t o5 = idct_limit((int32_t)descale<T>(t.t12 - t.o1, S));
    const uint32_t o3 = idct_limit((int32_t)descale<T>(t.t13 + t.o0, S));
    const uint32_t o4 = idct_limit((int32_t)descale<T>(t.t13 - t.o0, S));
    return (uint64_t)(o0 | (o1 << 8) | (o2 << 16) | (o3 << 24)) | ((uint64_t)(o4 | (o5 << 8) | (o6 << 16) | (o7 << 24)) << 32);
}

// coef: 64 zig-zag-order int16, q: 64 zig-zag-order quantisers (both 16-byte aligned);
// out: 8 rows of 8 samples (8-byte aligned rows, pitch `stride`).  jidctint.c jpeg_idct_islow:
// DEQUANTIZE in int (16 x 16 bits), both passes in JLONG, the workspace in int.
__host__ __device__ inline void idct_islow(const int16_t* coef, const int16_t* q, uint8_t* out, int64_t stride) {
    struct V16 { uint32_t w[4]; };
    union Blk { V16 v[8]; int16_t s[64]; } cz, qz;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        cz.v[i] = ((const V16*)coef)[i];
        qz.v[i] = ((const V16*)q)[i];
    }
    int32_t dq[64];
    uint32_t m1 = 0;
#pragma unroll
    for (int i = 0; i < 64; ++i) {   // natural order i = r * 8 + c
        dq[i] = (int32_t)cz.s[kZz[i]] * qz.s[kZz[i]];
        const uint32_t a = (uint32_t)(dq[i] < 0 ? -dq[i] : dq[i]);
        m1 = a > m1 ? a : m1;
    }
    int32_t ws[64];
    if (m1 <= (uint32_t)kPass1Max) idct_pass1<int32_t>(dq, ws);
    else idct_pass1<int64_t>(dq, ws);
    uint32_t m2 = 0;
#pragma unroll
    for (int i = 0; i < 64; ++i) {
        const uint32_t a = ws[i] < 0 ? 0u - (uint32_t)ws[i] : (uint32_t)ws[i];
        m2 = a > m2 ? a : m2;
    }
    const bool narrow = m2 <= (uint32_t)kPass2Max;
#pragma unroll
    for (int r = 0; r < 8; ++r)   // pass 2: rows
        *(uint64_t*)(out + r * stride) = narrow ? idct_row<int32_t>(ws + r * 8) : idct_row<int64_t>(ws + r * 8);
}

// ---------------------------------------------------------------- upsampling + colour
__host__ __device__ inline int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }
__host__ __device__ inline uint8_t clamp8(int v) { return (uint8_t)clampi(v, 0, 255); }

// One chroma sample of output pixel (x, y), component c with plane `pl` (pitch bw*8):
// jdsample.c h2v2_fancy_upsample / h2v1_fancy_upsample, or a plain copy at full resolution.
// Beyond the last downsampled column the triangle filter repeats the edge sample (libjpeg's
// special-cased first / last columns); rows above / below the component repeat the edge row
// (jdmainct.c context pointers).
__host__ __device__ inline int chroma_at(const JpegImage& im, const uint8_t* pl, int c, int x, int y) {
    const int64_t pitch = (int64_t)im.bw[c] * 8;
    const int hx = im.hs[0] / im.hs[c], vy = im.vs[0] / im.vs[c];
    if (hx == 1 && vy == 1) return pl[(int64_t)y * pitch + x];
    const int cx = x >> 1;
    const int dw = im.dw[c];
    // libjpeg-turbo's jinit_upsampler takes the fancy path only for downsampled_width > 2;
    // narrower components are replicated (h2v1_upsample / h2v2_upsample)
    if (dw <= 2) return pl[(int64_t)(vy == 2 ? y >> 1 : y) * pitch + cx];
    const int xn = (x & 1) ? (cx + 1 < dw ? cx + 1 : cx) : (cx > 0 ? cx - 1 : 0);
    if (vy == 1) {   // h2v1: (3 * this + neighbour + 1 or 2) >> 2
        const uint8_t* row = pl + (int64_t)y * pitch;
        return (3 * row[cx] + row[xn] + ((x & 1) ? 2 : 1)) >> 2;
    }
    // h2v2: column sums 3 * this row + nearer neighbouring row, then (3 * this + neighbour + 8 or 7) >> 4
    const int cy = y >> 1;
    const int yn = (y & 1) ? (cy + 1 < im.dh[c] ? cy + 1 : cy) : (cy > 0 ? cy - 1 : 0);
    const uint8_t* r0 = pl + (int64_t)cy * pitch;
    const uint8_t* r1 = pl + (int64_t)yn * pitch;
    const int s_this = 3 * r0[cx] + r1[cx];
    const int s_next = 3 * r0[xn] + r1[xn];
    return (3 * s_this + s_next + ((x & 1) ? 7 : 8)) >> 4;
}

// jdcolor.c ycc_rgb_convert with build_ycc_rgb_table's 16-bit fixed-point factors
__host__ __device__ inline void ycc_to_rgb(int yy, int cb, int cr, uint8_t* rgb) {
    constexpr int SB = 16;
    constexpr int32_t HALF = 1 << (SB - 1);
    const int32_t xb = cb - 128, xr = cr - 128;
    const int32_t r_off = (91881 * xr + HALF) >> SB;      // FIX(1.40200)
    const int32_t b_off = (116130 * xb + HALF) >> SB;     // FIX(1.77200)
    const int32_t g_off = ((-22554) * xb + HALF + (-46802) * xr) >> SB;   // FIX(0.34414), FIX(0.71414)
    rgb[0] = clamp8(yy + r_off);
    rgb[1] = clamp8(yy + g_off);
    rgb[2] = clamp8(yy + b_off);
}

// img_planes: this image's component planes (comp_plane[] relative to it)
__host__ __device__ inline void pixel_rgb(const JpegImage& im, const uint8_t* img_planes, int x, int y, uint8_t* rgb) {
    const uint8_t* p0 = img_planes + im.comp_plane[0];
    const int yy = p0[(int64_t)y * im.bw[0] * 8 + x];
    if (im.ncomp == 1) {
        rgb[0] = rgb[1] = rgb[2] = (uint8_t)yy;
        return;
    }
    const int c1 = chroma_at(im, img_planes + im.comp_plane[1], 1, x, y);
    const int c2 = chroma_at(im, img_planes + im.comp_plane[2], 2, x, y);
    if (im.cspace == CS_RGB) {
        rgb[0] = (uint8_t)yy;
        rgb[1] = (uint8_t)c1;
        rgb[2] = (uint8_t)c2;
    } else {
        ycc_to_rgb(yy, c1, c2, rgb);
    }
}

}  // namespace jpeg
}  // namespace reidmi
