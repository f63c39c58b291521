#!/usr/bin/env python3
"""Per-kernel durations and GPU idle gaps from a rocprofv3 --kernel-trace CSV.

usage: python tools/trace_gaps.py KERNEL_TRACE_CSV [NAME_SUBSTRING_OF_FIRST] [NAME_SUBSTRING_OF_LAST]

Reports, over the window from the first dispatch whose name holds the first
substring to the last one holding the second (default: the whole trace):
every kernel's calls / average / total duration, the busy time (union of the
dispatch intervals), the window and the idle fraction (the host not keeping
the queue fed), and the gap that follows each kernel (median / mean), which
names the launch that waits on the host."""
import csv
import statistics
import sys
from collections import defaultdict


def short(name):
    name = name.replace("void ", "").split("(")[0]
    return name if len(name) <= 60 else name[:57] + "..."


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])) for r in rows)
    a = sys.argv[2] if len(sys.argv) > 2 else None
    b = sys.argv[3] if len(sys.argv) > 3 else None
    i0 = next(i for i, e in enumerate(ev) if a is None or a in e[2])
    i1 = max(i for i, e in enumerate(ev) if b is None or b in e[2])
    ev = ev[i0: i1 + 1]
    per = defaultdict(list)
    gap_after = defaultdict(list)
    busy, cur_s, cur_e = 0, ev[0][0], ev[0][1]
    for k, (s, e, n) in enumerate(ev):
        per[n].append(e - s)
        if k + 1 < len(ev):
            gap_after[n].append(max(0, ev[k + 1][0] - e))
        if s > cur_e:
            busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    window = ev[-1][1] - ev[0][0]
    print(f"window {window / 1e6:.3f} ms, busy {busy / 1e6:.3f} ms, idle {100 * (1 - busy / window):.1f} %, "
          f"{len(ev)} dispatches")
    print(f"{'kernel':60s} {'calls':>6s} {'avg us':>8s} {'p10':>7s} {'p50':>7s} {'p90':>7s} {'tot ms':>8s} "
          f"{'gap after: med us':>18s} {'mean us':>8s}")
    for n, d in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        g = gap_after.get(n, [0])
        q = sorted(d)
        pct = [q[min(len(q) - 1, int(f * len(q)))] / 1e3 for f in (0.1, 0.5, 0.9)]
        print(f"{n:60s} {len(d):6d} {statistics.mean(d) / 1e3:8.2f} {pct[0]:7.2f} {pct[1]:7.2f} {pct[2]:7.2f} "
              f"{sum(d) / 1e6:8.3f} {statistics.median(g) / 1e3:18.2f} {statistics.mean(g) / 1e3:8.2f}")


if __name__ == "__main__":
    main()
