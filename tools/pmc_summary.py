"""Summarise tools/prof_round.sh's rocprofv3 --pmc passes (gpurun_out/ after a GPU call) into the
per-launch numbers DESIGN.md quotes: c_fc (M = BATCH x 211, N 3072, K 768) HBM-side bytes (FETCH_SIZE
x 2, the gfx950 wide-read correction of MI355X_MICROARCH.md "HBM", + WRITE_SIZE) against its
algorithmic bytes, per-dispatch duration / TF/s / the clock the chip held (GRBM_GUI_ACTIVE / 8 XCDs /
duration) / MFMA busy per SIMD (SQ_VALU_MFMA_BUSY_CYCLES / 1024 SIMDs / (SQ_BUSY_CYCLES / 32 SEs));
the vision attention (NSEQ 1024 x 12 heads, L = 211) likewise.

    python tools/pmc_summary.py [GPURUN_OUT] [BATCH]"""
import collections
import csv
import os
import statistics
import sys

PEAK = 2500.0  # TF/s at the 2.4 GHz nominal clock


def load(d, kernel):
    rows = list(csv.DictReader(open(os.path.join(d, "p_counter_collection.csv"))))
    agg = collections.defaultdict(float)
    span = {}
    for r in rows:
        if kernel not in r["Kernel_Name"]:
            continue
        i = int(r["Dispatch_Id"])
        agg[(i, r["Counter_Name"])] += float(r["Counter_Value"])
        span[i] = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
    out = collections.defaultdict(dict)
    for (i, c), v in agg.items():
        out[i][c] = v
    for i in out:
        out[i]["ns"] = span[i][1] - span[i][0]
    return dict(sorted(out.items()))


def main():
    root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
    batch = int(sys.argv[2]) if len(sys.argv) > 2 else 19281
    M = batch * 211
    cfc = "gemm_persistent_kernelILi1E"
    fl = 2.0 * M * 3072 * 768
    fetch = load(os.path.join(root, "pmc_FETCH_SIZE"), cfc)
    write = load(os.path.join(root, "pmc_WRITE_SIZE"), cfc)
    big = lambda d: [v for v in d.values() if v["ns"] > 1e6]  # noqa: E731 (full-size launches)
    f = statistics.median(v["FETCH_SIZE"] for v in big(fetch))
    w = statistics.median(v["WRITE_SIZE"] for v in big(write))
    alg = M * 768 * 2 + 3072 * 768 * 2 + M * 3072 * 2
    print(f"c_fc (M = {M}) traffic per launch: FETCH_SIZE {f:.0f} KiB (x2) + WRITE_SIZE {w:.0f} KiB = "
          f"{(2 * f + w) * 1024 / 1e9:.2f} GB; algorithmic {alg / 1e9:.2f} GB (A + W + out)")
    p2 = load(os.path.join(root, "cfc_pmc2"), cfc)
    for i, v in p2.items():
        if v["ns"] < 1e6:
            continue
        clk = v["GRBM_GUI_ACTIVE"] / 8 / v["ns"]  # GHz
        tfs = fl / v["ns"] / 1e3
        print(f"c_fc dispatch {i}: {v['ns'] / 1e3:.0f} us, {tfs:.0f} TF/s, clock {clk:.3f} GHz, "
              f"{tfs / (PEAK * clk / 2.4):.3f} of the peak at that clock")
    p1 = load(os.path.join(root, "cfc_pmc1"), cfc)
    for i, v in p1.items():
        if v["ns"] < 1e6:
            continue
        busy = v["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024 / (v["SQ_BUSY_CYCLES"] / 32)
        print(f"c_fc dispatch {i}: MFMA busy {busy:.3f}")
    at = "mhsa_pipe_kernel"
    nseq = int(os.environ.get("NSEQ", "1024"))
    a3 = load(os.path.join(root, "attn_pmc3"), at)
    a4 = load(os.path.join(root, "attn_pmc4"), at)
    a1 = load(os.path.join(root, "attn_pmc1"), at)
    if a3 and a4:
        f = statistics.median(v["FETCH_SIZE"] for v in a3.values())
        w = statistics.median(v["WRITE_SIZE"] for v in a4.values())
        ns = statistics.median(v["ns"] for v in a1.values())
        n = nseq * 12
        alg = n * 211 * 64 * 2 * 3 + n * 64 * 228 * 2
        hb = (2 * f + w) * 1024
        print(f"vision attention ({nseq} x 12 heads, L 211): {ns / 1e3:.0f} us, traffic {hb / 1e9:.3f} GB "
              f"(FETCH x2 + WRITE) against {alg / 1e9:.3f} GB algorithmic q / k / V^T / o "
              f"({hb / alg:.2f}x), {hb / ns:.0f} GB/s = {hb / ns / 8000:.2f} of 8 TB/s")


if __name__ == "__main__":
    main()
