#!/bin/bash
# Round-2 profiling pass (through gpurun from the repo root): rocprofv3 kernel
# trace + stats of the bench command (timed steps, no extra legs), and the PMC
# calibration lab under FETCH_SIZE and WRITE_SIZE (separate passes).  Each GPU
# step has its own limit; the script stops at the first failure.
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/prof2"
TAG="${1:-r02}"
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o "$TAG" \
    -- python3 "$ROOT/bench.py" --steps 10 --warmup 3 --no-extras > "$OUT/${TAG}_bench.json" 2> "$OUT/${TAG}_bench.err"
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/calib_fetch" -o calib \
    -- "$ROOT/tools/build/pmc_calib" > "$OUT/calib_expected.txt" 2>&1
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/calib_write" -o calib \
    -- "$ROOT/tools/build/pmc_calib" > /dev/null 2>&1
echo "prof done"
