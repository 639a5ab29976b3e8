"""Per-wave instruction budget of the persistent GEMM, per 256x256 tile, by section
(VERDICT r4 Next #5; DESIGN.md §5 "GEMM instruction budget").

    python tools/isa_budget.py [--asm FILE] [--pmc DIR[:M:N:K] ...]

Static: compiles multimodal-reid_amd/csrc/gemm.hip for gfx950 to assembly (or reads --asm) and,
for each <EPI, TAG> instance the encoders launch, counts instructions by class in the K-step loop
body (LLVM loop depth 2) and in the tile body (depth 1: K-step 0's issue plus the epilogue).
A tile is (K/64 - 1) K-step bodies + one tile body.  Static counts include both arms of the
partial-tile branches, so they bound the dynamic count from above.

Dynamic (optional): a rocprofv3 --pmc CSV directory holding SQ_INSTS_VALU / SQ_INSTS_SALU /
SQ_INSTS_MFMA / SQ_INSTS_LDS / SQ_WAVES for a GEMM of shape M x N x K (tools/prof_round.sh
passes *_pmc2); prints the per-wave per-tile counts that ran.  SQ_INSTS_VALU includes the MFMAs,
SQ_INSTS_LDS the LDS-DMA loads."""
import argparse
import collections
import csv
import glob
import os
import re
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "multimodal-reid_amd", "csrc")
INSTANCES = ((1, 0, "c_fc: LN-fold + QuickGELU, fp16 out", (768,)),
             (3, 0, "qkv: LN-fold, head-split Q/K/V^T stores", (768,)),
             (6, 0, "out_proj: bias + fp16 residual", (768,)),
             (6, 1, "c_proj: bias + fp16 residual", (3072,)))
KEYS = ("MFMA", "VALU", "TRANS", "SALU", "LDS", "DMA", "VMEM_LD", "VMEM_ST", "SYNC")


def cls(op):
    if op.startswith("v_mfma"):
        return "MFMA"
    if op.startswith(("v_exp", "v_rcp", "v_log", "v_rsq", "v_sqrt")):
        return "TRANS"
    if op.startswith("v_"):
        return "VALU"
    if op.startswith(("s_waitcnt", "s_barrier", "s_nop")):
        return "SYNC"
    if op.startswith("s_"):
        return "SALU"
    if op.startswith("ds_"):
        return "LDS"
    if op.startswith("global_load_lds"):
        return "DMA"
    if op.startswith(("global_load", "buffer_load", "scratch_load")):
        return "VMEM_LD"
    if op.startswith(("global_store", "buffer_store", "scratch_store")):
        return "VMEM_ST"
    return None


def assemble():
    out = os.path.join(tempfile.mkdtemp(), "gemm.s")
    subprocess.run(["hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-ffp-contract=off",
                    "-fhip-fp32-correctly-rounded-divide-sqrt", "-I.", "-I../../include", "--cuda-device-only",
                    "-S", "gemm.hip", "-o", out], cwd=CSRC, check=True)
    return out


def static_counts(lines, epi, tag):
    name = f"_ZN6reidmi22gemm_persistent_kernelILi{epi}ELi{tag}E"
    st = next(i for i, ln in enumerate(lines) if ln.startswith(name))
    en = next(i for i in range(st, len(lines)) if lines[i].startswith(".Lfunc_end"))
    depth, cnt = 0, {d: collections.Counter() for d in (0, 1, 2)}
    for raw in lines[st + 1:en]:
        code = raw.split(";")[0].strip()
        if code.endswith(":") and " " not in code:
            m = re.search(r"Depth=(\d+)", raw)
            depth = int(m.group(1)) if m else 0
            continue
        if not code or code.startswith("."):
            continue
        c = cls(code.split()[0])
        if c:
            cnt[min(depth, 2)][c] += 1
    return cnt


def pmc_counts(d):
    """{dispatch: {counter: value}} for the GEMM dispatches in a --pmc output directory."""
    per = collections.defaultdict(dict)
    for f in glob.glob(os.path.join(d, "**", "*.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "Counter_Name" in r and "gemm_persistent_kernel" in r["Kernel_Name"]:
                per[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
    return per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--asm")
    ap.add_argument("--pmc", action="append", default=[], help="DIR:M:N:K")
    a = ap.parse_args()
    lines = open(a.asm or assemble()).read().split("\n")
    print("static per-wave instruction counts, 256x256x64 tile, 8 waves (2 per SIMD)")
    for epi, tag, what, ks in INSTANCES:
        cnt = static_counts(lines, epi, tag)
        for K in ks:
            nk = K // 64
            tot = cnt[1] + collections.Counter({k: v * (nk - 1) for k, v in cnt[2].items()})
            print(f"<EPI {epi}, TAG {tag}> {what}, K = {K}")
            print("    per tile        " + " ".join(f"{k}={tot[k]}" for k in KEYS))
            print("    K-step body     " + " ".join(f"{k}={cnt[2][k]}" for k in KEYS))
            print("    tile body       " + " ".join(f"{k}={cnt[1][k]}" for k in KEYS) +
                  "   (K-step 0 issue + epilogue)")
    for spec in a.pmc:
        d, M, N, K = spec.split(":")
        M, N, K = int(M), int(N), int(K)
        tiles = -(-M // 256) * (N // 256)
        print(f"dynamic (SQ counters) {d}: M={M} N={N} K={K}, {tiles} tiles, per wave per tile")
        for disp, c in sorted(pmc_counts(d).items(), key=lambda t: int(t[0]))[-3:]:
            tw = tiles * 8
            mfma = c.get("SQ_INSTS_MFMA", 0)
            print(f"    dispatch {disp}: MFMA={mfma / tw:.0f} VALU(non-MFMA)={(c.get('SQ_INSTS_VALU', 0) - mfma) / tw:.0f} "
                  f"SALU={c.get('SQ_INSTS_SALU', 0) / tw:.0f} LDS+DMA={c.get('SQ_INSTS_LDS', 0) / tw:.0f} "
                  f"VMEM={c.get('SQ_INSTS_VMEM', 0) / tw:.0f}")


if __name__ == "__main__":
    sys.exit(main())
