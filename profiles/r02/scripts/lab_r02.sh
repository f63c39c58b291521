#!/bin/bash
# Round-2 labs on the GPU box (through gpurun): KL speculation A/B, device
# Laplacian build kernel trace.  Each step has its own limit; stop on failure.
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/lab2"
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 python3 "$ROOT/tools/kl_spec_lab.py" > "$OUT/kl_spec.txt" 2>&1
cat "$OUT/kl_spec.txt"
EK_TRACE=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/build" -o build \
    -- python3 "$ROOT/tools/build_lab.py" > "$OUT/build.txt" 2>&1
grep -E "device=|spmv_setup_pins" "$OUT/build.txt" | head -30
head -20 "$OUT/build/build_kernel_stats.csv" | cut -c1-150
