"""Print a rocprofv3 --stats kernel summary (every *kernel_stats.csv under DIR):
calls, average and total duration per kernel.  usage: python tools/kstats.py DIR [top]"""
import csv
import glob
import sys

top = int(sys.argv[2]) if len(sys.argv) > 2 else 14
for path in sorted(glob.glob(f"{sys.argv[1]}/**/*kernel_stats.csv", recursive=True)):
    print(path)
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
    for r in rows[:top]:
        name = r["Name"].split("(")[0].replace("ek::dev::", "").replace("(anonymous namespace)::", "")[:48]
        print(f"  {name:48s} {int(r['Calls']):7d} {float(r['AverageNs']) / 1e3:10.2f} us {float(r['TotalDurationNs']) / 1e6:9.2f} ms")
