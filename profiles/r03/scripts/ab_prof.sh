#!/bin/bash
# GPU box: rocprofv3 kernel stats of the headline file steps, parked build
# (tools/build/wip) against the in-tree one, alternated.
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/ab_prof"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for v in new old new old; do
  ( if [ $v = old ]; then export EK_LIB_PATH="$ROOT/tools/build/wip/libeigkl_hip.so"; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$v" -o run \
      -- python3 "$ROOT/tools/spmv_probe.py" file 1.15lcc 1 1 3 > "$OUT/$v.txt" 2>&1 ) || exit 3
  echo "== $v"
  python3 -c "
import csv
for r in list(csv.DictReader(open('$OUT/$v/run_kernel_stats.csv')))[:4]: print(f\"{r['Name'][:40]:40s} {int(r['Calls']):6d} {float(r['AverageNs'])/1000:9.3f} us\")"
done
