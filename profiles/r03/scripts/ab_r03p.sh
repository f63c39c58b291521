#!/bin/bash
# GPU box: gemm_vq XCD remap; TT=0/1 wall A/B (round 3)
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
cd "$ROOT"
bash tools/gpu_tests.sh r03p tests/test_gpu_parity.py -k "device_paths or golden"
REPS=5 timeout -k 10 300 python tools/lanczos_ab.py 1,10 - EK_LANCZOS_TT=0 > "$OUT/r03p_ab.txt" 2>&1
cat "$OUT/r03p_ab.txt"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/r03p_prof10" -o run \
    -- python3 "$ROOT/tools/lanczos_ab.py" 10 - > "$OUT/r03p_prof10.txt" 2>&1
echo done
