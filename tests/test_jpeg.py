"""JPEG decode (data_prepare.py:87-92: `Image.open(path).convert("RGB")` in the loader
workers).  The decoder the reference runs is Pillow 12.2 on libjpeg-turbo, importable here
and on the GPU box, so it is the oracle: reidmi_jpeg_decode must reproduce its RGB output
bit for bit.  CPU tests cover the host-side plan (statuses, layout, table pooling); GPU tests
decode on the device."""
import io

import numpy as np
import pytest
import torch
from PIL import Image

from multimodal_reid_amd import data_prepare
from multimodal_reid_amd import synthetic as syn


def pil_rgb(b):
    return np.asarray(Image.open(io.BytesIO(b)).convert("RGB"))


def _gray(h, w, seed, **kw):
    g = io.BytesIO()
    Image.fromarray(syn.crop_rgb(h, w, seed)[:, :, 0]).save(g, "JPEG", **kw)
    return g.getvalue()


def _save(arr, **kw):
    b = io.BytesIO()
    Image.fromarray(arr).save(b, "JPEG", **kw)
    return b.getvalue()


def _dht(tc_th, lengths, symbols):
    """A DHT segment: BITS from the code-length counts, HUFFVAL in canonical order."""
    body = bytes([tc_th]) + bytes(lengths[1:17]) + bytes(symbols)
    return b"\xff\xc4" + (2 + len(body)).to_bytes(2, "big") + body


def _stuff(bits):
    """Entropy-coded segment from a '0'/'1' string (padded with 1s), 0xFF stuffed as FF 00."""
    bits += "1" * (-len(bits) % 8)
    out = bytearray()
    for i in range(0, len(bits), 8):
        out.append(int(bits[i:i + 8], 2))
        if out[-1] == 0xFF:
            out.append(0)
    return bytes(out)


def stuffed_window_cases():
    """Hand-built grayscale baseline files whose entropy data puts two stuffed pairs
    (FF 00 FF 00) in one 4-byte refill window while the bit window holds only 5 bits, followed
    by a 16-bit AC code and 10 extra bits (the word path of BitReader::refill used to
    return with 21 bits, and the extra bits read zeros).  Custom tables: DC category 0 = '0',
    category c = '1' + 15 zeros; AC codes of every length 2..16 on a '0 1...1 0' ladder, EOB =
    '00', run/size 0x0A = '0' + 15 ones.  Variants shift the window state with the DC category
    (bits left 5 / 1 / 9) and with a second FF 00 pair right after the first window."""
    dqt = b"\xff\xdb\x00\x43\x00" + bytes([1] * 64)
    ac_len = [0] * 17
    for L in range(2, 16):
        ac_len[L] = 1
    ac_len[16] = 3
    # EOB, 13 fillers (lengths 3..15), then the three 16-bit codes: A, B = '0' + 15 ones (0x0A), C
    ac_sym = [0x00] + list(range(0x11, 0x1B)) + [0x31, 0x32, 0x33] + [0x21, 0x0A, 0x22]
    ac_b = "0" + "1" * 15
    out = []
    for name, cat, extra, tail, second in (("ffff-b5", 11, "01111111111", "1111111111", False),
                                           ("ffff-b1", 15, "011111111111111", "1111111111", False),
                                           ("ffff-b9", 7, "0111111", "1111111110", False),
                                           ("ffff-b5-twice", 11, "01111111111", "1111111111", True)):
        dc_len = [0] * 17
        dc_len[1], dc_len[16] = 1, 1
        blocks = 8
        bits = "1" + "0" * 15 + extra + ac_b + tail   # block 0: DC category `cat`, one AC coefficient
        if second:   # a second coefficient with the same 16-bit code: FF 00 FF 00 once more
            bits += ac_b + "1" * 10
        bits += "00" + "000" * (blocks - 1)           # EOB; blocks 1..: DC diff 0, EOB
        sof = b"\xff\xc0\x00\x0b\x08\x00\x08" + (8 * blocks).to_bytes(2, "big") + b"\x01\x01\x11\x00"
        sos = b"\xff\xda\x00\x08\x01\x01\x00\x00\x3f\x00"
        f = (b"\xff\xd8" + dqt + sof + _dht(0x00, dc_len, [0, cat]) + _dht(0x10, ac_len, ac_sym) + sos
             + _stuff(bits) + b"\xff\xd9")
        assert b"\xff\x00\xff\x00" in f
        out.append((name, f))
    return out


def parity_cases():
    """Edge geometry (1 px, narrow chroma that libjpeg-turbo replicates instead of filtering,
    partial MCUs), every Pillow subsampling, low / high quality, restart intervals, optimised
    Huffman tables, grayscale, Adobe-RGB-free YCbCr — all Pillow-encoded."""
    out = []
    sizes = [(128, 64), (1, 1), (2, 2), (3, 5), (4, 3), (17, 33), (15, 2), (2, 15), (64, 128), (200, 97), (31, 1),
             (9, 8), (16, 16), (33, 17)]
    for i, (h, w) in enumerate(sizes):
        for ss in (0, 1, 2):
            for q in (30, 75, 97):
                out.append((f"{h}x{w}-ss{ss}-q{q}", syn.jpeg_files(1, h, w, seed=i, quality=q, subsampling=ss,
                                                                    offset=ss * 10 + q)[0]))
    out.append(("rst-blocks", syn.jpeg_files(1, 128, 64, seed=3, restart_marker_blocks=3)[0]))
    out.append(("rst-rows", syn.jpeg_files(1, 77, 45, seed=4, restart_marker_rows=1)[0]))
    out.append(("rst-444", syn.jpeg_files(1, 50, 70, seed=5, subsampling=0, restart_marker_blocks=1)[0]))
    out.append(("optimize", syn.jpeg_files(1, 128, 64, seed=6, optimize=True)[0]))
    out.append(("optimize-422", syn.jpeg_files(1, 99, 41, seed=7, optimize=True, subsampling=1)[0]))
    out.append(("q100-444", syn.jpeg_files(1, 128, 64, seed=8, quality=100, subsampling=0)[0]))
    out.append(("q1", syn.jpeg_files(1, 128, 64, seed=9, quality=1)[0]))
    out.append(("flat", _save(np.full((40, 24, 3), 77, np.uint8), quality=90)))
    out.append(("extremes", _save(np.where(np.indices((64, 32)).sum(0)[..., None] % 2 == 0, 0, 255)
                                  .astype(np.uint8).repeat(3, 2), quality=100, subsampling=0)))
    out.append(("gray", _gray(37, 29, 7, quality=85)))
    out.append(("gray-rst", _gray(128, 64, 8, quality=60, restart_marker_blocks=2)))
    return out + stuffed_window_cases()


# ------------------------------------------------------------------ CPU: host plan


def test_plan_status_and_meta():
    good = syn.jpeg_files(3, 128, 64, seed=1)
    prog = _save(syn.crop_rgb(32, 16, 2), progressive=True)
    cmyk = io.BytesIO()
    Image.fromarray(syn.crop_rgb(16, 16, 3)).convert("CMYK").save(cmyk, "JPEG")
    files = [good[0], b"not a jpeg", prog, good[1], cmyk.getvalue(), good[2][:40], _gray(5, 7, 4)]
    jb = data_prepare.JpegBatch(files)
    assert jb.status.tolist() == [0, 1, 2, 0, 3, 1, 0]
    assert jb.meta.tolist() == [[0, 128, 64], [0, 0, 0], [0, 0, 0], [128 * 64 * 3, 128, 64], [0, 0, 0], [0, 0, 0],
                                [2 * 128 * 64 * 3, 5, 7]]
    assert int(jb.info[5]) == 4 and jb.out_bytes == 2 * 128 * 64 * 3 + 5 * 7 * 3
    assert (jb.max_h, jb.max_w) == (128, 64)
    with pytest.raises(ValueError, match="4 of 7"):
        jb.raise_for_status()


def _segments(b):
    """(marker, offset, length) of the header segments up to SOS."""
    p, out = 2, []
    while p < len(b):
        m, n = b[p + 1], (b[p + 2] << 8) | b[p + 3]
        out.append((m, p, n))
        if m == 0xDA:
            break
        p += 2 + n
    return out


def _pil_raises(b):
    try:
        pil_rgb(b)
    except OSError:
        return True
    return False


def corrupt_header_cases():
    """Header damage libjpeg rejects (Pillow raises) and one table form the device does not
    take: (name, bytes, expected plan status)."""
    good = syn.jpeg_files(1, 128, 64, seed=21)[0]
    seg = _segments(good)
    out = []
    b = bytearray(good)   # a component names quantisation table 5 (jdinput.c: JERR_NO_QUANT_TABLE)
    p = next(p for m, p, _ in seg if m == 0xC0)
    b[p + 4 + 8] = 5
    out.append(("tq5", bytes(b), 4))
    b = bytearray(good)   # DC table with two 1-bit codes (jdhuff.c: JERR_BAD_HUFF_TABLE)
    p = next(p for m, p, _ in seg if m == 0xC4) + 4
    assert b[p] >> 4 == 0 and b[p + 3] >= 2
    b[p + 1] += 2
    b[p + 3] -= 2
    out.append(("huff-overfull", bytes(b), 4))
    b = bytearray(good)   # DC table symbol 16 (a DC category above 15)
    p = next(p for m, p, _ in seg if m == 0xC4) + 4
    b[p + 17] = 16
    out.append(("huff-dc-symbol", bytes(b), 4))
    # a 16-bit quantisation table with an entry above 32767 (libjpeg keeps UINT16): unsupported
    p, n = next((p, n) for m, p, n in seg if m == 0xDB)
    q = good[p + 5:p + 5 + 64]
    t16 = bytes([0x10]) + b"".join(int(v).to_bytes(2, "big") for v in q)
    t16 = t16[:3] + (40000).to_bytes(2, "big") + t16[5:]
    seg16 = b"\xff\xdb" + (2 + len(t16)).to_bytes(2, "big") + t16
    out.append(("dqt16-big", good[:p] + seg16 + good[p + 2 + n:], 2))
    return out


def test_plan_rejects_corrupt_headers_like_libjpeg():
    cases = corrupt_header_cases()
    jb = data_prepare.JpegBatch([b for _, b, _ in cases])
    assert jb.status.tolist() == [st for _, _, st in cases]
    for name, b, st in cases:
        if st == 4:   # the reference's loader fails on these too
            assert _pil_raises(b), name


def truncated_cases():
    good = syn.jpeg_files(2, 128, 64, seed=22)
    return [("mid-scan", good[0][:int(len(good[0]) * 0.6)]), ("no-eoi", good[1][:-2])]


def tail_cases():
    """Files whose scan is followed by something other than EOI: trailing bytes
    with no EOI, a lone 0xFF, another marker, a cut inside the last bytes — with and without
    restart intervals, several sizes and subsamplings.  Pillow (the reference's decoder,
    libjpeg-turbo 3.1 behind a suspending source) loads some and raises for others; what
    decides it is whether libjpeg's bit-buffer fetches reach the end of the data before the
    last MCU (jpeg_core.h LjInput), and which marker follows the scan."""
    out = []
    for i, (h, w, sub, q, kw) in enumerate([(64, 48, 2, 90, {}), (128, 64, 2, 90, {}), (37, 29, 1, 75, {}),
                                            (128, 64, 0, 95, {}), (200, 150, 2, 50, {}), (16, 16, 2, 90, {}),
                                            (128, 64, 2, 90, {"restart_marker_blocks": 4}),
                                            (96, 80, 1, 80, {"restart_marker_rows": 1}), (300, 200, 2, 92, {})]):
        body = syn.jpeg_files(1, h, w, seed=40 + i, quality=q, subsampling=sub, **kw)[0][:-2]
        for extra in (b"", b"\x00", b"\x00" * 2, b"\x00" * 3, b"\x00" * 4, b"\x00" * 5, b"\x00" * 6, b"\x00" * 9,
                      b"\x12\x34\x56\x78\x9a", b"\xff", b"\xff\xd9", b"\xff\xd8", b"\xff\xd0", b"\xff\xfe\x00\x02"):
            out.append((f"{i}+{extra.hex()}", body + extra))
        for cut in (1, 2, 3, 5, 17, 100):
            if cut < len(body) - 700:
                out.append((f"{i}-{cut}", body[:-cut]))
    return out + marker_tail_cases()


def _marker_segments(rng):
    """Marker segments libjpeg's read_markers may meet after the scan (jdmarker.c), valid and
    damaged: parameterless markers, SOI / SOFn / JPG / reserved, SOS headers (whole, cut, bad
    length or component selectors), DQT / DHT / DAC / DRI with good and bad lengths and indices,
    APPn / COM / DNL with short lengths, garbage, 0xFF fill and stuffing."""
    import struct

    def rb(k):
        return bytes(rng.randrange(256) for _ in range(k))

    def u16(v):
        return struct.pack(">H", v)

    ch = rng.choice
    return [b"\xff\xd9", b"\xff\xd8", b"\xff\xd0", b"\xff\x01", b"\xff\xda", b"\xff\xc0", b"\xff\xc2", b"\xff\xc8",
            b"\xff\xde", b"\xff\xf0", b"\xff\xcc",
            b"\xff\xfe" + u16(ch([0, 1, 2, 3, 4, 8])) + rb(ch([0, 1, 2, 6])),
            b"\xff" + bytes([rng.randrange(0xE0, 0xF0)]) + u16(ch([0, 1, 2, 4, 16])) + b"ab",
            b"\xff\xdb" + u16(ch([2, 3, 67, 68, 131, 60, 132, 100])) + bytes([ch([0, 1, 4, 0x10, 0x13, 0x20])])
            + bytes(rng.randrange(1, 256) for _ in range(ch([0, 10, 64, 65, 128, 129]))),
            b"\xff\xc4" + u16(ch([2, 19, 20, 21, 30, 18])) + bytes([ch([0, 1, 0x10, 0x13, 5, 0x15, 0x20])])
            + bytes([ch([0, 1, 2, 3])] + [0] * 15) + rb(ch([0, 1, 2, 3])),
            b"\xff\xcc" + u16(ch([2, 4, 6, 5, 3])) + bytes(rng.randrange(40) for _ in range(ch([0, 2, 4]))),
            b"\xff\xdd" + u16(ch([4, 5, 3])) + b"\x00\x00",
            b"\xff\xdc" + u16(ch([4, 2, 0])) + b"\x00\x10",
            b"\xff\xda" + u16(ch([12, 8, 13, 10])) + bytes([ch([3, 1, 0, 2, 5])])
            + bytes([ch([1, 2, 3, 9]), 0x11, ch([1, 2, 3]), 0x11, ch([3, 1]), 0x11, 0, 63, 0])[:ch(range(10))],
            rb(ch([1, 2, 3])), b"\xff", b"\xff\x00", b"\xff\xff\xd9", b"\xff\xff\xd8"]


def marker_tail_cases(n=240, seed=5):
    """What follows a complete scan, as libjpeg's jpeg_finish_decompress reads it:
    SOS after a single-scan image, markers after COM / APPn / tables, DQT / DHT / DAC / DRI
    contents, sequences cut anywhere.  Seeded random sequences of 1-4 segments after two bodies
    (4:2:0 and 4:2:2) plus the advisor's named cases; Pillow decides which load."""
    import random
    rng = random.Random(seed)
    bodies = [syn.jpeg_files(1, 64, 48, seed=40)[0][:-2], syn.jpeg_files(1, 37, 29, seed=42, subsampling=1)[0][:-2]]
    com = b"\xff\xfe\x00\x04ab"
    sos = b"\xff\xda\x00\x0c\x03\x01\x00\x02\x11\x03\x11\x00\x3f\x00"
    out = [("sos", bodies[0] + sos), ("sos-cut", bodies[0] + sos[:5]), ("com+sos", bodies[0] + com + sos),
           ("com+soi", bodies[0] + com + b"\xff\xd8"), ("com+sof", bodies[0] + com + b"\xff\xc0\x00\x11"),
           ("com+eoi+soi", bodies[0] + com + b"\xff\xd9\xff\xd8"), ("ffda", bodies[1] + b"\xff\xda")]
    for k in range(n):
        body = bodies[k % 2]
        tail = b"".join(rng.choice(_marker_segments(rng)) for _ in range(rng.choice([1, 2, 3, 4])))
        b = body + tail
        if rng.random() < 0.3 and len(tail) > 1:
            b = b[:len(body) + rng.randrange(1, len(tail))]
        out.append((f"m{k}:{b[len(body):][:24].hex()}", b))
    return out

def _mutations(files, n, seed):
    """Random damage of whole files: cuts anywhere, bit flips, overwritten byte runs, inserted
    0xFF / marker bytes."""
    r = np.random.default_rng(seed)
    out = []
    for k in range(n):
        b = bytearray(files[k % len(files)])
        kind = k % 4
        if kind == 0:
            b = b[:int(r.integers(1, len(b)))]
        elif kind == 1:
            for _ in range(int(r.integers(1, 8))):
                i = int(r.integers(0, len(b)))
                b[i] ^= 1 << int(r.integers(0, 8))
        elif kind == 2:
            i = int(r.integers(0, len(b)))
            m = int(r.integers(1, 16))
            b[i:i + m] = bytes(r.integers(0, 256, m, dtype=np.uint8))
        else:
            i = int(r.integers(2, len(b)))
            b[i:i] = bytes([0xFF, int(r.choice([0x00, 0xD0, 0xD8, 0xD9, 0xDA, 0xC4, 0xDB, 0xDD, 0xFE, 0xFF]))])
        out.append(bytes(b))
    return out


def damaged_cases(n=400, seed=7):
    """Damaged files: random cuts, bit flips, overwritten runs and inserted 0xFF / marker bytes
    (headers and scans alike) of 4:2:0, restart-interval and 4:2:2 files."""
    seeds = syn.jpeg_files(6, 128, 64, seed=61) + syn.jpeg_files(2, 77, 45, seed=62, restart_marker_rows=1) + \
        syn.jpeg_files(2, 37, 29, seed=63, subsampling=1)
    return _mutations(seeds, n, seed)


_PIL_C_PATH = """
import io, sys, numpy as np
from PIL import Image
d = np.load(sys.argv[1], allow_pickle=False)
out = {}
for k in range(int(d["n"])):
    try:
        out[f"i{k}"] = np.asarray(Image.open(io.BytesIO(d[f"f{k}"].tobytes())).convert("RGB"))
    except Exception:
        pass
np.savez(sys.argv[2], **out)
"""


def pillow_c_path(files, tmp_path):
    """Pillow's decode of each file (None where it raises) with libjpeg-turbo's SIMD off
    (JSIMD_FORCENONE=1, a fresh process): libjpeg's C islow IDCT.  Pillow's default SIMD islow
    works in 16-bit lanes and differs from the C definition only for coefficients far outside
    any encoder's range (damaged data); on valid files the two are bit-identical."""
    import subprocess
    import sys
    src, dst = tmp_path / "files.npz", tmp_path / "pil.npz"
    np.savez(src, n=len(files), **{f"f{k}": np.frombuffer(b, np.uint8) for k, b in enumerate(files)})
    import os
    subprocess.run([sys.executable, "-c", _PIL_C_PATH, str(src), str(dst)], check=True,
                   env=dict(os.environ, JSIMD_FORCENONE="1"))
    d = np.load(dst, allow_pickle=False)
    return [d[f"i{k}"] if f"i{k}" in d.files else None for k in range(len(files))]


def test_plan_pools_tables_and_reads_paths(tmp_path):
    files = syn.jpeg_files(20, 128, 64, seed=2)   # one encoder setting: one set of tables
    for i, b in enumerate(files[:3]):
        (tmp_path / f"{i}.jpg").write_bytes(b)
    jb = data_prepare.JpegBatch(files)
    hdr = jb.plan[:72].view(np.int64)   # JpegPlan: B, n_huff, n_quant, ...
    assert hdr[0] == 20 and hdr[1] == 4 and hdr[2] == 2
    jp = data_prepare.JpegBatch([tmp_path / f"{i}.jpg" for i in range(3)])
    assert np.array_equal(jp.buf, np.frombuffer(b"".join(files[:3]), np.uint8))
    assert jp.status.tolist() == [0, 0, 0]
    empty = data_prepare.JpegBatch([])
    assert empty.B == 0 and empty.out_bytes == 0


def test_core_arithmetic_on_host_vs_pillow(tmp_path):
    """jpeg_core.h (the kernels' per-image decode, IDCT and colour code) compiled for the host
    by tools/jpeg_host_check.hip and run serially over parity_cases(): equal to Pillow."""
    import ctypes
    import os
    import shutil
    import subprocess
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    if not shutil.which(hipcc):
        pytest.skip("hipcc not available")
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    so = str(tmp_path / "libjpeghost.so")
    subprocess.run([hipcc, "-O2", "-std=c++17", "-fPIC", "-shared", f"-I{repo}/multimodal-reid_amd/csrc",
                    f"-I{repo}/include", f"{repo}/tools/jpeg_host_check.hip", "-o", so], check=True)
    host = ctypes.CDLL(so)
    cases = parity_cases()
    jb = data_prepare.JpegBatch([b for _, b in cases])
    out = np.zeros(jb.out_bytes, np.uint8)
    err = np.zeros(jb.B, np.int32)
    vp = ctypes.c_void_p
    host.jpeg_host_decode(jb.buf.ctypes.data_as(vp), jb.plan.ctypes.data_as(vp), jb.info.ctypes.data_as(vp),
                          out.ctypes.data_as(vp), err.ctypes.data_as(vp))
    assert not err.any()
    # files that end before EOI: status 6, where Pillow raises "image file is truncated"
    tc = truncated_cases()
    jt = data_prepare.JpegBatch([b for _, b in tc])
    assert not jt.status.any()   # the headers are whole
    tout = np.zeros(max(jt.out_bytes, 1), np.uint8)
    terr = np.zeros(jt.B, np.int32)
    host.jpeg_host_decode(jt.buf.ctypes.data_as(vp), jt.plan.ctypes.data_as(vp), jt.info.ctypes.data_as(vp),
                          tout.ctypes.data_as(vp), terr.ctypes.data_as(vp))
    assert terr.tolist() == [6] * len(tc)
    assert all(_pil_raises(b) for _, b in tc)
    # after the scan: the device decoder returns an image exactly when Pillow does
    ec = tail_cases()
    je = data_prepare.JpegBatch([b for _, b in ec])
    eout = np.zeros(max(je.out_bytes, 1), np.uint8)
    eerr = np.zeros(je.B, np.int32)
    host.jpeg_host_decode(je.buf.ctypes.data_as(vp), je.plan.ctypes.data_as(vp), je.info.ctypes.data_as(vp),
                          eout.ctypes.data_as(vp), eerr.ctypes.data_as(vp))
    # the kernels' decode-only first pass (replay only where the end of the data decides) gives
    # the statuses and pixels of replaying libjpeg's input buffering for every image
    rout = np.zeros_like(eout)
    rerr = np.zeros_like(eerr)
    host.jpeg_host_decode_replay(je.buf.ctypes.data_as(vp), je.plan.ctypes.data_as(vp), je.info.ctypes.data_as(vp),
                                 rout.ctypes.data_as(vp), rerr.ctypes.data_as(vp))
    assert np.array_equal(eerr, rerr) and np.array_equal(eout, rout)
    mism = [(name, int(eerr[k])) for k, (name, b) in enumerate(ec) if (eerr[k] == 0) == _pil_raises(b)]
    assert not mism, mism
    assert 0 < int((eerr == 0).sum()) < len(ec)  # both kinds occur
    for k, (name, b) in enumerate(ec):  # and the images it returns are Pillow's pixels
        if eerr[k] == 0:
            off, h, w = je.meta[k]
            assert np.array_equal(eout[off:off + h * w * 3].reshape(h, w, 3), pil_rgb(b)), name
    bad = [name for i, (name, b) in enumerate(cases)
           if not np.array_equal(out[jb.meta[i, 0]:jb.meta[i, 0] + jb.meta[i, 1] * jb.meta[i, 2] * 3]
                                 .reshape(jb.meta[i, 1], jb.meta[i, 2], 3), pil_rgb(b))]
    assert not bad, bad
    # damaged files (headers and scans): the same files load, with libjpeg's C-path pixels
    dm = damaged_cases()
    jd = data_prepare.JpegBatch(dm)
    dout = np.zeros(max(jd.out_bytes, 1), np.uint8)
    derr = np.zeros(jd.B, np.int32)
    host.jpeg_host_decode(jd.buf.ctypes.data_as(vp), jd.plan.ctypes.data_as(vp), jd.info.ctypes.data_as(vp),
                          dout.ctypes.data_as(vp), derr.ctypes.data_as(vp))
    _check_damaged(dm, np.where(jd.status != 0, jd.status, derr), jd.meta, dout, pillow_c_path(dm, tmp_path))


def _check_damaged(files, status, meta, pix, ref):
    """status 0 exactly where Pillow returns an image (J_LAYOUT aside: sampling layouts the
    device does not decode raise too), and then Pillow's C-path pixels."""
    bad = []
    for k, b in enumerate(files):
        if status[k] == 3:
            continue
        if (status[k] == 0) != (ref[k] is not None):
            bad.append((k, int(status[k]), ref[k] is not None))
        elif status[k] == 0:
            off, h, w = meta[k]
            if not np.array_equal(pix[off:off + h * w * 3].reshape(h, w, 3), ref[k]):
                bad.append((k, "pixels"))
    assert not bad, bad
    assert 100 < int((status == 0).sum()) and ((status == 5).any() or (status == 6).any())


# ------------------------------------------------------------------ GPU: device decode vs Pillow


@pytest.mark.gpu
def test_decode_bitexact_vs_pillow(gpu):
    cases = parity_cases()
    pix, meta, jb = data_prepare.decode_jpeg([b for _, b in cases])
    torch.cuda.synchronize()
    pix = pix.cpu().numpy()
    bad = []
    for i, (name, b) in enumerate(cases):
        off, h, w = jb.meta[i]
        got = pix[off:off + h * w * 3].reshape(h, w, 3)
        if not np.array_equal(got, pil_rgb(b)):
            bad.append(name)
    assert not bad, bad
    assert np.array_equal(meta.cpu().numpy(), jb.meta)


@pytest.mark.gpu
def test_decode_market_batch_bitexact(gpu):
    """A Market-1501-shaped batch (128 x 64, 4:2:0) of 1500 files in one call, every image
    equal to Pillow's decode."""
    files = syn.jpeg_files(1500, 128, 64, seed=11, quality=90)
    pix, _, jb = data_prepare.decode_jpeg(files)
    got = pix.cpu().numpy().reshape(1500, 128, 64, 3)
    ref = np.stack([pil_rgb(b) for b in files])
    assert np.array_equal(got, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.float16])
def test_preprocess_jpeg_equals_pil_pipeline(gpu, dtype):
    """decode -> Resize(256, 128) -> ToTensor -> Normalize from the JPEG bytes equals the same
    transform applied to Pillow-decoded images (itself pinned to Pillow, test_transforms.py)."""
    files = syn.jpeg_files(40, 128, 64, seed=12) + [syn.jpeg_files(1, 300, 110, seed=13, subsampling=1)[0],
                                                    _gray(97, 41, 14, quality=80)]
    a = data_prepare.preprocess_jpeg(files, dtype=dtype)
    b = data_prepare.preprocess([Image.open(io.BytesIO(f)) for f in files], dtype=dtype)
    assert torch.equal(a.view(torch.int16 if dtype == torch.float16 else torch.int32),
                       b.view(torch.int16 if dtype == torch.float16 else torch.int32))


@pytest.mark.gpu
def test_decode_rejects_unsupported_and_reports_bad_data(gpu):
    prog = _save(syn.crop_rgb(32, 16, 2), progressive=True)
    with pytest.raises(ValueError, match="progressive"):
        data_prepare.decode_jpeg([syn.jpeg_files(1, 8, 8)[0], prog])
    # a corrupted entropy segment: the device pass flags it (status 5) or decodes garbage the
    # way libjpeg does, never faults; unchecked decode still returns the good images intact
    good = syn.jpeg_files(2, 64, 32, seed=15)
    bad = bytearray(good[1])
    sos = bytes(bad).find(b"\xff\xda")
    for k in range(sos + 20, len(bad) - 2, 7):
        bad[k] = 0xFF if bad[k + 1] == 0 else bad[k] ^ 0x5A
    pix, _, jb = data_prepare.decode_jpeg([good[0], bytes(bad)], check=False)
    torch.cuda.synchronize()
    got = pix.cpu().numpy()[:64 * 32 * 3].reshape(64, 32, 3)
    assert np.array_equal(got, pil_rgb(good[0]))


@pytest.mark.gpu
def test_decode_damaged_files_vs_pillow(gpu, tmp_path):
    """The device decode of damaged files (cuts, bit flips, overwritten runs, inserted markers in
    headers and scans): an image exactly where Pillow returns one, with libjpeg's C-path pixels."""
    dm = damaged_cases(400, 8)
    pix, _, jb, err = data_prepare.decode_jpeg(dm, check=False, return_status=True)
    torch.cuda.synchronize()
    st = np.where(jb.status != 0, jb.status, err.cpu().numpy()[:len(dm)])
    _check_damaged(dm, st, jb.meta, pix.cpu().numpy(), pillow_c_path(dm, tmp_path))


@pytest.mark.gpu
def test_decode_reports_truncated_files(gpu):
    """A file that ends inside the scan, or lacks only its EOI, is reported (status 6) where
    the reference's Image.open(...).convert("RGB") raises; the other files of the batch decode."""
    tc = truncated_cases()
    good = syn.jpeg_files(1, 40, 24, seed=23)[0]
    with pytest.raises(ValueError, match="truncated"):
        data_prepare.decode_jpeg([good] + [b for _, b in tc])
    pix, _, jb = data_prepare.decode_jpeg([good] + [b for _, b in tc], check=False)
    torch.cuda.synchronize()
    assert np.array_equal(pix.cpu().numpy()[:40 * 24 * 3].reshape(40, 24, 3), pil_rgb(good))
    # what follows the scan (no EOI, trailing bytes, another marker): the device decoder returns
    # an image exactly when Pillow does, with Pillow's pixels
    ec = tail_cases()
    pix, _, jb, err = data_prepare.decode_jpeg([b for _, b in ec], check=False, return_status=True)
    torch.cuda.synchronize()
    err, pix = err.cpu().numpy()[:len(ec)], pix.cpu().numpy()
    for k, (name, b) in enumerate(ec):
        assert (err[k] == 0) != _pil_raises(b), name
        if err[k] == 0:
            off, h, w = jb.meta[k]
            assert np.array_equal(pix[off:off + h * w * 3].reshape(h, w, 3), pil_rgb(b)), name
