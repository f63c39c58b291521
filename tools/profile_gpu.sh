#!/bin/bash
# GPU-box profiling recipe (run through gpurun from the repo root):
#   1. SpMV layout lab
#   2. rocprofv3 kernel trace + stats of the default bench workload
#   3. PMC passes for the HBM traffic of the same command, one counter group
#      per pass (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950)
# Every GPU step has its own time limit; the script stops at the first failure.
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/prof"
TAG="${1:-r01}"
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
BENCH=(python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-sweep)
if [ -x "$ROOT/tools/build/spmv_lab" ]; then
    timeout -k 10 120 "$ROOT/tools/build/spmv_lab" 1.0 200 > "$OUT/${TAG}_spmv_lab.txt" 2>&1
fi
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o "$TAG" \
    -- "${BENCH[@]}" > "$OUT/${TAG}_bench_trace.log" 2>&1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o "$TAG" \
    -- "${BENCH[@]}" > "$OUT/${TAG}_pmc_fetch.log" 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o "$TAG" \
    -- "${BENCH[@]}" > "$OUT/${TAG}_pmc_write.log" 2>&1
echo "profile done"
