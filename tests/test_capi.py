"""CPU-side checks of the drop-in boundary: libreidmi.so loads and exports every entry
point include/reidmi.h declares, and the ctypes table in _lib.py covers them all; the tools
library (include/reidmi_tools.h) adds exactly its forced-variant entry points, which the
product library does not export.  No compute calls (no GPU here)."""
import ctypes
import os
import re

import pytest

from conftest import REPO

HEADER = os.path.join(REPO, "include", "reidmi.h")
TOOLS_HEADER = os.path.join(REPO, "include", "reidmi_tools.h")
LIB = os.path.join(REPO, "multimodal-reid_amd", "libreidmi.so")
TOOLS_LIB = os.path.join(REPO, "multimodal-reid_amd", "libreidmi_tools.so")


def declared(header=HEADER):
    txt = open(header).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(reidmi_\w+)\s*\(", txt)))


def test_header_declares_entry_points():
    names = declared()
    assert "reidmi_distmat_f32" in names and "reidmi_eval_rows" in names
    assert len(names) >= 6


def test_library_exports_every_declared_symbol():
    if not os.path.exists(LIB):
        pytest.skip("libreidmi.so not built (run __graft_entry__.build())")
    import torch  # noqa: F401  (load torch's HIP runtime first, as the product does)
    L = ctypes.CDLL(LIB)
    missing = [n for n in declared() if not hasattr(L, n)]
    assert not missing, missing
    L.reidmi_abi_version.restype = ctypes.c_int
    assert L.reidmi_abi_version() >= 1


def test_ctypes_table_matches_header():
    from multimodal_reid_amd import _lib
    names = set(declared()) - {"reidmi_last_error", "reidmi_abi_version"}
    covered = set(_lib.SIGNATURES) | set(_lib.STRUCT_ENTRY_POINTS)
    assert names == covered, names ^ covered


def test_tools_library_exports_variants_product_does_not():
    if not (os.path.exists(LIB) and os.path.exists(TOOLS_LIB)):
        pytest.skip("libraries not built (run __graft_entry__.build())")
    import torch  # noqa: F401
    from multimodal_reid_amd import _lib
    tools = declared(TOOLS_HEADER)
    assert set(tools) == set(_lib.TOOLS_SIGNATURES)
    assert not set(tools) & set(declared())
    P, T = ctypes.CDLL(LIB), ctypes.CDLL(TOOLS_LIB)
    assert not [n for n in tools if hasattr(P, n)], "the product library must not export the A/B variants"
    missing = [n for n in tools + declared() if not hasattr(T, n)]
    assert not missing, missing


@pytest.mark.parametrize("src,define", [("gemm.hip", "-DGEMM_VAR_NOSTORE=1"), ("gemm.hip", "-DGEMM_VAR_FB2=0"),
                                        ("gemm.hip", "-DGEMM_VAR_NODMA=1"),
                                        ("backend.hip", "-DDM2_BK_=32"), ("backend.hip", "-DRS_STATS")])
def test_variant_macros_refused_outside_tools_builds(src, define):
    """The A/B timing hooks (some compile kernels with wrong results by design) are an #error
    unless the tools define is set, so no variant can be built into libreidmi.so."""
    import shutil
    import subprocess
    from multimodal_reid_amd import build_lib as B
    if not shutil.which(B.HIPCC):
        pytest.skip("hipcc not available")
    base = [B.HIPCC, "-E", "-x", "hip", "--offload-arch=gfx950", "--cuda-device-only", f"-I{B.CSRC}",
            f"-I{B.INCLUDE}", os.path.join(B.CSRC, src), "-o", os.devnull]
    bad = subprocess.run(base + [define], capture_output=True, text=True)
    assert bad.returncode != 0 and "REIDMI_TOOLS" in bad.stderr
    ok = subprocess.run(base + [define, B.TOOLS_DEFINE], capture_output=True, text=True)
    assert ok.returncode == 0, ok.stderr[-2000:]


# the encoder's GEMM instances (EPI 0-6).  The re-rank pre-filter's EPI_RRHI / EPI_RRSV (7, 8)
# spill 20 bytes per lane in the tile prologue, where each reload is followed by the compiler's
# own vmcnt(0) (an over-wait: safe; their K-loops keep the plain vmcnt(6), no deferred stores)
_GEMM_ENCODER = tuple(f"gemm_persistent_kernelILi{e}E" for e in range(7))


@pytest.mark.parametrize("src,kernels", [("attention.hip", ("mhsa_kernel", "mhsa_pipe_kernel")),
                                         ("gemm.hip", _GEMM_ENCODER)])
def test_counted_wait_kernels_use_no_scratch(src, kernels):
    """The kernels whose `s_waitcnt vmcnt(N)` counts are derived from their own vector-memory
    instructions (attention's K/V^T rings, the GEMM's deferred epilogue stores) must not spill:
    a scratch load or store would enter the same counter and let a wait return early.
    Checked on the compiler's resource report of the product build flags."""
    import shutil
    import subprocess
    from multimodal_reid_amd import build_lib as B
    if not shutil.which(B.HIPCC):
        pytest.skip("hipcc not available")
    flags = [f for f in B.FLAGS if f not in ("-fPIC", "-fno-gpu-rdc")]
    r = subprocess.run([B.HIPCC, *flags, "--cuda-device-only", "-c", "-Rpass-analysis=kernel-resource-usage",
                        os.path.join(B.CSRC, src), "-o", os.devnull], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    name, seen = None, 0
    for line in r.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            name = m.group(1)
            continue
        m = re.search(r"ScratchSize \[bytes/lane\]: (\d+)", line)
        if m and name and any(k in name for k in kernels):
            seen += 1
            assert int(m.group(1)) == 0, f"{name} spills to scratch ({m.group(1)} bytes/lane)"
    assert seen >= 3, r.stderr[-2000:]
