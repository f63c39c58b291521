#!/bin/bash
# Lab (run through gpurun): bench line + rocprofv3 kernel-trace summary of the
# default workload, for A/B of kernel changes.  Writes gpurun_out/quick/.
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/quick"
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 120 python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-sweep > "$OUT/bench.json"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o q \
    -- python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-sweep > "$OUT/trace.log" 2>&1
echo done
