#!/bin/bash
# GPU box: LDS-staged column reduce A/B (round 3)
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
cd "$ROOT"
bash tools/gpu_tests.sh r03o tests/test_gpu_parity.py tests/test_multirank_gpu.py -k "device_paths or golden or multirank or sharded"
timeout -k 10 300 python tools/lanczos_ab.py 1,2,10 EK_UPD_RED=1 EK_UPD_RED=0 EK_LANCZOS_TT=0 > "$OUT/r03o_ab.txt" 2>&1
cat "$OUT/r03o_ab.txt"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/r03o_prof10" -o run \
    -- python3 "$ROOT/tools/lanczos_ab.py" 10 - > "$OUT/r03o_prof10.txt" 2>&1
EK_UPD_RED=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/r03o_prof1_red0" -o run \
    -- python3 "$ROOT/tools/lanczos_ab.py" 1 - > "$OUT/r03o_prof1_red0.txt" 2>&1
EK_LANCZOS_TT=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/r03o_prof1_tt0" -o run \
    -- python3 "$ROOT/tools/lanczos_ab.py" 1 - > "$OUT/r03o_prof1_tt0.txt" 2>&1
echo done
