"""Builds libreidmi.so in-tree from csrc/*.hip with hipcc for gfx950.

Plain shared library with a C ABI (include/reidmi.h): no torch headers, no
pybind.  It links libamdhip64.so.7 by soname, so inside a process that already
imported torch it binds to the HIP runtime torch loaded (one runtime, shared
streams)."""
import concurrent.futures as cf
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, "csrc")
OBJ = os.path.join(PKG, "build")
LIB = os.path.join(PKG, "libreidmi.so")
INCLUDE = os.path.join(os.path.dirname(PKG), "include")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-ffp-contract=off",
         "-fhip-fp32-correctly-rounded-divide-sqrt", "-fno-gpu-rdc", "-Wno-unused-result",
         f"-I{CSRC}", f"-I{INCLUDE}"]


def _sources():
    return sorted(f for f in os.listdir(CSRC) if f.endswith(".hip"))


def _headers_mtime():
    hs = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    hs += [os.path.join(INCLUDE, f) for f in os.listdir(INCLUDE) if f.endswith(".h")] if os.path.isdir(INCLUDE) else []
    return max([os.path.getmtime(h) for h in hs] + [os.path.getmtime(__file__)])


def _compile(src):
    obj = os.path.join(OBJ, src.replace(".hip", ".o"))
    srcp = os.path.join(CSRC, src)
    if os.path.exists(obj) and os.path.getmtime(obj) > max(os.path.getmtime(srcp), _headers_mtime()):
        return obj, False
    cmd = [HIPCC, *FLAGS, "-c", srcp, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr[-6000:]}")
    return obj, True


def build(verbose=False, jobs=None):
    os.makedirs(OBJ, exist_ok=True)
    jobs = jobs or min(8, os.cpu_count() or 4, 16)
    with cf.ThreadPoolExecutor(jobs) as ex:
        res = list(ex.map(_compile, _sources()))
    objs = [o for o, _ in res]
    changed = any(c for _, c in res)
    if changed or not os.path.exists(LIB) or os.path.getmtime(LIB) < max(os.path.getmtime(o) for o in objs):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB, *objs]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr[-4000:]}")
        if verbose:
            print("built", LIB)
    return LIB


if __name__ == "__main__":
    build(verbose=True)
    sys.exit(0)
