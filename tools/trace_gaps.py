import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
ev = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name']) for r in rows)
t0 = ev[0][0]
segs = []; cur = [ev[0]]
for e in ev[1:]:
    if e[0] - cur[-1][1] > 20e6: segs.append(cur); cur = [e]
    else: cur.append(e)
segs.append(cur)
for s in segs:
    wall = (s[-1][1] - s[0][0]) / 1e6; busy = sum(e[1] - e[0] for e in s) / 1e6
    gaps = sorted(((b[0] - a[1]) / 1e3, a[2][:50], b[2][:50]) for a, b in zip(s, s[1:]))[-5:]
    print("seg %.3f s wall %.1f ms busy %.1f ms (%.1f%%) n=%d" % ((s[0][0] - t0) / 1e9, wall, busy, 100 * busy / wall, len(s)))
    for g in gaps: print("   gap %.1f us after %s before %s" % g)
