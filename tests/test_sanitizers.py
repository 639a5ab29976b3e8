"""The CPU code that parses untrusted bytes or indexes by data-dependent bounds, run under
AddressSanitizer + UndefinedBehaviorSanitizer (VERDICT r4 Next #7):

* the C restatement (oracle/reid_oracle.c, transforms_oracle.c) through oracle/asan_driver.c:
  the oracle tests' own inputs (the golden fixtures' features, tie-heavy distances, junk and
  distractor labels, the re-rank fixture's distances at k1 = 50 / 20, Pillow resize shapes) and
  edge cases (one-item galleries, queries with no match, wide k1 / k2), 1 and 4 threads;
* the JPEG host code — the header parser reidmi_jpeg_plan (jpeg.hip) and jpeg_core.h's
  per-image decode, marker walk, IDCT and colour conversion (tools/jpeg_asan_main.hip) — over
  the parity cases, the truncated / tail / marker cases, and random cuts, bit flips and byte
  overwrites of fixture files.

Both are standalone executables built by `make -C oracle asan` (every sanitizer report is
fatal, so a clean exit is the check); each answer is also compared with the unsanitised build
(liboracle.so, libreidmi.so + the host decode), so the sanitised runs execute the same paths."""
import ctypes
import os
import shutil
import struct
import subprocess

import numpy as np
import pytest

import oracle
from conftest import REPO, golden
from multimodal_reid_amd import synthetic as syn

ASAN_DIR = os.path.join(REPO, "oracle", "build", "asan")
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:halt_on_error=1",
           UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")


@pytest.fixture(scope="module")
def asan_bins():
    if not shutil.which("make") or not shutil.which(os.environ.get("CC", "gcc")):
        pytest.skip("no C toolchain")
    r = subprocess.run(["make", "-C", os.path.join(REPO, "oracle"), "asan"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    return os.path.join(ASAN_DIR, "oracle_asan"), os.path.join(ASAN_DIR, "jpeg_asan")


class _Batch:
    """Calls for oracle_asan (protocol in oracle/asan_driver.c) and their expected answers."""

    def __init__(self):
        self.req, self.expect = [], []

    def add(self, op, params, arrays, expect):
        self.req.append(struct.pack("<ii", op, len(params)) + struct.pack(f"<{len(params)}q", *params))
        self.req += [np.ascontiguousarray(a).tobytes() for a in arrays]
        self.expect.append(expect)

    def run(self, exe):
        r = subprocess.run([exe], input=b"".join(self.req) + struct.pack("<ii", -1, 0), capture_output=True,
                           env=ENV, timeout=600)
        assert r.returncode == 0, r.stderr.decode(errors="replace")[-4000:]
        out, pos = r.stdout, 0
        for exp in self.expect:
            for e in exp:
                n = e.nbytes
                got = np.frombuffer(out[pos:pos + n], dtype=e.dtype).reshape(e.shape)
                pos += n
                assert np.array_equal(got.view(np.uint8), np.ascontiguousarray(e).view(np.uint8))
        assert pos == len(out)


def _eval_expect(d, qp, gp, qc, gc):
    v, f, a, n = oracle.eval_rows(d, qp, gp, qc, gc)
    return [v.astype(np.int32), f, a, n]


def _i64(a):
    return np.ascontiguousarray(a, np.int64)


def test_oracle_under_asan_ubsan(asan_bins):
    b = _Batch()
    for threads in (1, 4):
        b.add(7, [threads], [], [])
        oracle.set_threads(threads)
        # the backend fixture's inputs (tests/test_oracle.py): normalise, distance, top-k, eval
        qp, gp, qc, gc = syn.labels(100, 500, num_ids=60, num_cams=6, seed=1, distractor_frac=0.1, junk_frac=0.04)
        qf, gf = syn.features(qp, gp, dim=1280, seed=1, noise=4.0)
        feats = np.concatenate([qf, gf])
        n = oracle.l2norm(feats)
        b.add(0, [600, 1280], [feats], [n])
        d = oracle.distmat(n[:100], n[100:])
        b.add(1, [100, 500, 1280], [n[:100], n[100:]], [d])
        for k in (1, 50, 500):
            b.add(2, [100, 500, k], [d], [oracle.topk_rows(d, k)])
        b.add(3, [100, 500], [d, _i64(qp), _i64(gp), _i64(qc), _i64(gc)], [_eval_expect(d, qp, gp, qc, gc)][0])
        # tie-heavy distances (backend_ties.npz) and edge cases: no match, one gallery item
        t = golden("backend_ties.npz")
        args = [t["distmat"], t["q_pids"], t["g_pids"], t["q_cams"], t["g_cams"]]
        b.add(3, list(t["distmat"].shape), [args[0]] + [_i64(a) for a in args[1:]], _eval_expect(*args))
        r = np.random.default_rng(threads)
        d1 = r.random((7, 1)).astype(np.float32)
        e_args = [d1, np.arange(7), np.array([3]), np.zeros(7), np.ones(1)]
        b.add(3, [7, 1], [d1] + [_i64(a) for a in e_args[1:]], _eval_expect(*e_args))
        dn = r.random((5, 40)).astype(np.float32)
        n_args = [dn, np.full(5, 99), np.arange(40) % 7, np.zeros(5), np.arange(40) % 3]
        b.add(3, [5, 40], [dn] + [_i64(a) for a in n_args[1:]], _eval_expect(*n_args))
        # the re-rank fixture's distances (rerank_small.npz), k1/k2 of evaluate.py:126 and a wide k1 = 120, k2 = 40
        rr = golden("rerank_small.npz")
        D = np.ascontiguousarray(rr["dist_all"], np.float32)
        for (k1, k2, Q) in ((50, 15, 100), (20, 6, 100), (120, 40, 30)):
            N = D.shape[0]
            fin, rank, vqe, jac = oracle.rerank_from_dist(D, Q, k1, k2, 0.3, debug=True)
            lam_h = int(np.float16(0.7).view(np.uint16))
            lam_f = int(np.float32(0.3).view(np.uint32))
            b.add(4, [N, Q, k1, k2, lam_h, lam_f], [D], [fin, rank, vqe, jac])
        # Pillow resize / ToTensor+Normalize shapes (transforms_oracle.c)
        for (h, w, oh, ow) in ((128, 64, 256, 128), (1, 1, 256, 128), (300, 97, 256, 128), (256, 128, 256, 128),
                               (5, 700, 3, 2)):
            img = r.integers(0, 256, (h, w, 3), dtype=np.uint8)
            b.add(5, [h, w, oh, ow], [img], [oracle.pil_resize(img, oh, ow)])
            mean = np.array([0.5, 0.4, 0.3], np.float32)
            std = np.array([0.2, 0.5, 0.7], np.float32)
            b.add(6, [h, w], [img, mean, std], [oracle.to_tensor_normalize(img, mean, std)])
    oracle.set_threads(1)
    b.run(asan_bins[0])


def test_jpeg_host_code_under_asan_ubsan(asan_bins, tmp_path):
    from multimodal_reid_amd import build_lib
    from multimodal_reid_amd.data_prepare import JpegBatch
    from test_jpeg import damaged_cases, parity_cases, tail_cases, truncated_cases
    base = [b for _, b in parity_cases()] + [b for _, b in truncated_cases()] + [b for _, b in tail_cases()]
    files = base + damaged_cases(400, 7) + [b"", b"\xff", b"\xff\xd8", b"\xff\xd8\xff"]
    # the unsanitised reference: libreidmi's plan + the host decode (as test_jpeg.py builds it)
    so = str(tmp_path / "libjpeghost.so")
    subprocess.run([build_lib.HIPCC, "-O2", "-std=c++17", "-fPIC", "-shared", f"-I{build_lib.CSRC}",
                    f"-I{build_lib.INCLUDE}", os.path.join(REPO, "tools", "jpeg_host_check.hip"), "-o", so], check=True)
    host = ctypes.CDLL(so)
    jb = JpegBatch(files)
    vp = ctypes.c_void_p
    ref_out = np.zeros(max(jb.out_bytes, 1), np.uint8)
    ref_err = np.zeros(jb.B, np.int32)
    host.jpeg_host_decode(jb.buf.ctypes.data_as(vp), jb.plan.ctypes.data_as(vp), jb.info.ctypes.data_as(vp),
                          ref_out.ctypes.data_as(vp), ref_err.ctypes.data_as(vp))
    blob = struct.pack("<q", len(files)) + np.asarray(jb.offsets, np.int64).tobytes() + jb.buf.tobytes()
    r = subprocess.run([asan_bins[1]], input=blob, capture_output=True, env=ENV, timeout=600)
    assert r.returncode == 0, r.stderr.decode(errors="replace")[-4000:]
    B, out = len(files), r.stdout
    st = np.frombuffer(out, np.int32, B, 0)
    meta = np.frombuffer(out, np.int64, 3 * B, 4 * B).reshape(B, 3)
    info = np.frombuffer(out, np.int64, 10, 4 * B + 24 * B)
    o = 4 * B + 24 * B + 80
    err = np.frombuffer(out, np.int32, B, o)
    err_replay = np.frombuffer(out, np.int32, B, o + 4 * B)
    pix = np.frombuffer(out, np.uint8, int(info[2]), o + 8 * B)
    assert np.array_equal(st, jb.status) and np.array_equal(meta, jb.meta) and np.array_equal(info, jb.info)
    assert np.array_equal(err, ref_err) and np.array_equal(err, err_replay)
    okm = err == 0
    assert np.array_equal(pix[:jb.out_bytes], ref_out[:jb.out_bytes])
    print(f"jpeg under ASan/UBSan: {B} files, plan statuses {np.bincount(st).tolist()}, decode statuses "
          f"{np.bincount(err).tolist()}, {int(okm.sum())} decoded")
    assert int(okm.sum()) > 100 and (err == 6).any() and (err == 5).any()
