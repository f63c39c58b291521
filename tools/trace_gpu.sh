#!/bin/bash
# rocprofv3 kernel-trace summary of the default bench workload (run through gpurun)
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
TAG="${1:-trace}"
OUT="$ROOT/gpurun_out/prof"
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$TAG" -o "$TAG" \
    -- python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-sweep >"$OUT/${TAG}.log" 2>&1
python3 - "$OUT/$TAG/${TAG}_kernel_stats.csv" <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:14]:
    print(f"{r['Name'][:70]:70s} {int(r['Calls']):6d} {float(r['AverageNs'])/1e3:9.2f} us {float(r['Percentage']):6.2f}%")
PY
