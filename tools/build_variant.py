"""Build an A/B variant of libreidmi.so: one source recompiled with extra -D flags, linked
with the in-tree objects of the others -> tools/variants/libreidmi_<name>.so.  The source is
compiled with -DREIDMI_TOOLS (the variant macros are an #error without it).

    python tools/build_variant.py NAME SOURCE.hip -DFOO=1 [-DBAR=2 ...]"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multimodal-reid_amd"))
import build_lib as B  # noqa: E402


def main():
    name, src, defs = sys.argv[1], sys.argv[2], sys.argv[3:]
    B.build()
    out_dir = os.path.join(ROOT, "tools", "variants")
    os.makedirs(out_dir, exist_ok=True)
    obj = os.path.join(out_dir, f"{name}_{src.replace('.hip', '.o')}")
    # -DREIDMI_TOOLS: the variant macros are refused without it (gemm.hip / backend.hip #error)
    r = subprocess.run([B.HIPCC, *B.FLAGS, B.TOOLS_DEFINE, *defs, "-c", os.path.join(B.CSRC, src), "-o", obj],
                       capture_output=True, text=True)
    if r.returncode:
        sys.exit(r.stderr[-4000:])
    objs = [obj if f == src else os.path.join(B.OBJ, f.replace(".hip", ".o")) for f in B._sources()]
    lib = os.path.join(out_dir, f"libreidmi_{name}.so")
    r = subprocess.run([B.HIPCC, f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-o", lib, *objs],
                       capture_output=True, text=True)
    if r.returncode:
        sys.exit(r.stderr[-4000:])
    print("built", lib)


if __name__ == "__main__":
    main()
