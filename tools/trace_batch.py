"""Per-kernel durations of one encoder batch from a rocprofv3 --kernel-trace CSV:
    python tools/trace_batch.py <kernel_trace.csv> [batch index]"""
import csv
import sys


def main():
    r = list(csv.DictReader(open(sys.argv[1])))
    nb = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    seq = sorted((int(x["Start_Timestamp"]), int(x["End_Timestamp"]), x["Kernel_Name"][:60]) for x in r)
    ims = [j for j, s in enumerate(seq) if "im2col" in s[2]]
    a, b = ims[nb], ims[nb + 1]
    busy = sum(seq[j][1] - seq[j][0] for j in range(a, b))
    print(f"batch {nb}: {b - a} kernels, wall {(seq[b][0] - seq[a][0]) / 1e3:.1f} us, busy {busy / 1e3:.1f} us")
    for j in range(a, min(b, a + 16)):
        print(f"{(seq[j][1] - seq[j][0]) / 1e3:9.1f}  {seq[j][2]}")


if __name__ == "__main__":
    main()
