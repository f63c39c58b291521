#!/bin/bash
# Round-3 profiling pass (through gpurun from the repo root): the rocprofv3
# kernel trace + stats of the same child command bench.py times its roofline
# from (tools/spmv_probe.py file 1.15lcc 1 1 3: the headline workload), and of
# the 10x resident solve.
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
TAG="${1:-r03}"
OUT="$ROOT/gpurun_out/prof3"
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace1x" -o "$TAG" \
    -- python3 "$ROOT/tools/spmv_probe.py" file 1.15lcc 1 1 3 > "$OUT/${TAG}_1x.txt" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace10x" -o "$TAG" \
    -- python3 "$ROOT/tools/spmv_probe.py" resident 10.0 10 > "$OUT/${TAG}_10x.txt" 2>&1
echo "prof done"
