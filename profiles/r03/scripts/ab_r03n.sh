#!/bin/bash
# GPU box: alpha hand-off batching + update reduction A/B (round 3)
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
cd "$ROOT"
bash tools/gpu_tests.sh r03n tests/test_gpu_parity.py -k "device_paths or golden or panel or three_term"
timeout -k 10 300 python tools/lanczos_ab.py 1,2,10 EK_UPD_RED=1 EK_UPD_RED=0 EK_LANCZOS_TT=0,EK_UPD_RED=0 > "$OUT/r03n_ab.txt" 2>&1
cat "$OUT/r03n_ab.txt"
cd /tmp
export TMPDIR=/tmp
for red in 1 0; do
  EK_UPD_RED=$red timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/r03n_prof_red$red" -o run \
      -- python3 "$ROOT/tools/lanczos_ab.py" 1 - > "$OUT/r03n_prof_red$red.txt" 2>&1
  EK_UPD_RED=$red timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/r03n_prof10_red$red" -o run \
      -- python3 "$ROOT/tools/lanczos_ab.py" 10 - > "$OUT/r03n_prof10_red$red.txt" 2>&1
done
echo done
