"""Builds libreidmi.so in-tree from csrc/*.hip with hipcc for gfx950.

Plain shared library with a C ABI (include/reidmi.h): no torch headers, no
pybind.  It links libamdhip64.so.7 by soname, so inside a process that already
imported torch it binds to the HIP runtime torch loaded (one runtime, shared
streams).

Rebuilds are decided by content, not by file times: every object records the sha256 of its
source, the headers and the compiler flags, and the library is written together with
libreidmi.manifest.json (the same digests).  _lib.load() refuses a library whose manifest
does not match the sources next to it, so a stale or foreign libreidmi.so cannot be used
silently, and the manifest says which sources a given library was built from.

libreidmi_tools.so (include/reidmi_tools.h) is the product library plus the forced-variant
entry points that tests and A/B tools use: the sources that hold `#ifdef REIDMI_TOOLS`
sections are compiled a second time with -DREIDMI_TOOLS (build/tools/) and linked with the
product objects of the other sources.  The product library never contains those sections."""
import concurrent.futures as cf
import hashlib
import json
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, "csrc")
OBJ = os.path.join(PKG, "build")
LIB = os.path.join(PKG, "libreidmi.so")
MANIFEST = os.path.join(PKG, "libreidmi.manifest.json")
TOOLS_LIB = os.path.join(PKG, "libreidmi_tools.so")
TOOLS_MANIFEST = os.path.join(PKG, "libreidmi_tools.manifest.json")
TOOLS_DEFINE = "-DREIDMI_TOOLS"
INCLUDE = os.path.join(os.path.dirname(PKG), "include")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-ffp-contract=off",
         "-fhip-fp32-correctly-rounded-divide-sqrt", "-fno-gpu-rdc", "-Wno-unused-result",
         f"-I{CSRC}", f"-I{INCLUDE}"]
LDFLAGS = [f"--offload-arch={ARCH}", "-shared", "-fPIC", "-ldl"]


def _flags_key():
    """The compiler/linker flags with the include paths made relative (the GPU box runs the
    tree from another directory)."""
    rel = [f if not f.startswith("-I") else "-I" + os.path.relpath(f[2:], PKG) for f in FLAGS]
    return " ".join(rel + LDFLAGS)


def _sources():
    return sorted(f for f in os.listdir(CSRC) if f.endswith(".hip"))


def _headers():
    hs = sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h"))
    if os.path.isdir(INCLUDE):
        hs += sorted(os.path.join(INCLUDE, f) for f in os.listdir(INCLUDE) if f.endswith(".h"))
    return hs


def _sha(path):
    with open(path, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def source_digests():
    """{relative path: sha256} of every input of the library (sources, headers, flags)."""
    d = {os.path.relpath(os.path.join(CSRC, s), PKG): _sha(os.path.join(CSRC, s)) for s in _sources()}
    d.update({os.path.relpath(h, PKG): _sha(h) for h in _headers()})
    d["flags"] = hashlib.sha256(_flags_key().encode()).hexdigest()
    return d


def _headers_digest():
    h = hashlib.sha256()
    for p in _headers():
        h.update(os.path.basename(p).encode())
        h.update(_sha(p).encode())
    h.update(_flags_key().encode())
    return h.hexdigest()


def _tools_sources():
    """Sources with a REIDMI_TOOLS section (compiled twice)."""
    return [s for s in _sources() if "REIDMI_TOOLS" in open(os.path.join(CSRC, s)).read()]


def _compile(src, hdr, tools=False):
    odir = os.path.join(OBJ, "tools") if tools else OBJ
    obj = os.path.join(odir, src.replace(".hip", ".o"))
    stamp = obj + ".sha256"
    srcp = os.path.join(CSRC, src)
    key = hashlib.sha256((_sha(srcp) + hdr + (TOOLS_DEFINE if tools else "")).encode()).hexdigest()
    if os.path.exists(obj) and os.path.exists(stamp) and open(stamp).read().strip() == key:
        return obj, False
    cmd = [HIPCC, *FLAGS, *([TOOLS_DEFINE] if tools else []), "-c", srcp, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr[-6000:]}")
    with open(stamp, "w") as f:
        f.write(key)
    return obj, True


def manifest_matches(tools=False):
    """True when the library exists and its manifest records exactly the current sources."""
    lib, man = (TOOLS_LIB, TOOLS_MANIFEST) if tools else (LIB, MANIFEST)
    if not (os.path.exists(lib) and os.path.exists(man)):
        return False
    try:
        with open(man) as f:
            m = json.load(f)
    except (OSError, ValueError):
        return False
    return m.get("inputs") == source_digests() and m.get("lib_sha256") == _sha(lib)


def _link(lib, man, objs, res, tools, verbose):
    changed = any(c for _, c in res)
    if not changed and manifest_matches(tools):
        if verbose:
            print("up to date", lib)
        return
    # the tools library binds its own copies of the internal symbols (a process may load both)
    cmd = [HIPCC, *LDFLAGS, *(["-Wl,-Bsymbolic"] if tools else []), "-o", lib, *objs]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr[-4000:]}")
    ver = subprocess.run([HIPCC, "--version"], capture_output=True, text=True).stdout.strip().splitlines()
    with open(man, "w") as f:
        json.dump({"inputs": source_digests(), "lib_sha256": _sha(lib), "arch": ARCH, "tools": tools,
                   "compiler": ver[0] if ver else "", "rebuilt": [os.path.basename(o) for o, c in res if c]},
                  f, indent=1, sort_keys=True)
    if verbose:
        print("built", lib, "(recompiled:", ", ".join(os.path.basename(o) for o, c in res if c) or "none", ")")


def build(verbose=False, jobs=None, tools=True):
    os.makedirs(os.path.join(OBJ, "tools"), exist_ok=True)
    jobs = jobs or min(8, os.cpu_count() or 4, 16)
    hdr = _headers_digest()
    srcs = _sources()
    tsrcs = _tools_sources() if tools else []
    jobs_list = [(s, False) for s in srcs] + [(s, True) for s in tsrcs]
    with cf.ThreadPoolExecutor(jobs) as ex:
        allres = list(ex.map(lambda st: _compile(st[0], hdr, st[1]), jobs_list))
    res = allres[:len(srcs)]
    _link(LIB, MANIFEST, [o for o, _ in res], res, False, verbose)
    if tools:
        tres = allres[len(srcs):]
        tobj = {s: r for s, r in zip(tsrcs, tres)}
        tres_all = [tobj.get(s, r) for s, r in zip(srcs, res)]
        _link(TOOLS_LIB, TOOLS_MANIFEST, [o for o, _ in tres_all], tres_all, True, verbose)
    return LIB


if __name__ == "__main__":
    build(verbose=True)
    sys.exit(0)
