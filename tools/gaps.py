"""Idle gaps between consecutive kernels of a rocprofv3 kernel trace
(*kernel_trace.csv under DIR): total kernel time, total gap time and the gap
histogram, per window of the trace between host-visible pauses > 2 ms.
usage: python tools/gaps.py DIR"""
import csv
import glob
import sys

for path in sorted(glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True)):
    rows = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(path))))
    segs, cur = [], [rows[0]]
    for r in rows[1:]:
        if r[0] - cur[-1][1] > 2_000_000:
            segs.append(cur)
            cur = [r]
        else:
            cur.append(r)
    segs.append(cur)
    print(path)
    for sg in segs:
        if len(sg) < 100:
            continue
        busy = sum(e - s for s, e, _ in sg) / 1e6
        gaps = [sg[i + 1][0] - sg[i][1] for i in range(len(sg) - 1)]
        span = (sg[-1][1] - sg[0][0]) / 1e6
        big = sorted(gaps)[-5:]
        print(f"  {len(sg):6d} kernels span {span:8.3f} ms busy {busy:8.3f} ms idle {span - busy:7.3f} ms; "
              f"gaps>20us {sum(1 for g in gaps if g > 20000)} ({sum(g for g in gaps if g > 20000) / 1e6:.3f} ms); "
              f"largest {[round(g / 1e3, 1) for g in big]} us")
