#!/bin/bash
# A/B of a parked library build (tools/build/wip: libeigkl_hip.so and, when
# present, its test_gpu_parity.py) against the in-tree build, through gpurun
# from the repo root: Lanczos restart A/B and the parked build's parity tests.
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out"
cd "$ROOT"
WIP="$ROOT/tools/build/wip/libeigkl_hip.so"
for v in main wip; do
  if [ $v = wip ]; then export EK_LIB_PATH=$WIP; else unset EK_LIB_PATH; fi
  timeout -k 10 300 python -u tools/restart_ab.py - > "$OUT/abw_restart_$v.txt" 2>&1 || exit 4
  sed "s/^/$v /" "$OUT/abw_restart_$v.txt"
  EK_LANCZOS_TRACE=1 timeout -k 10 100 python -u tools/lanczos_trace.py 2>&1 | grep factorization | sed "s/^/$v /"
done
export EK_LIB_PATH=$WIP
[ -f tools/build/wip/test_gpu_parity_wip.py ] && cp tools/build/wip/test_gpu_parity_wip.py tests/test_gpu_parity.py
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "lanczos or lcc or basis32 or panel or solve" > "$OUT/abw_tests.log" 2>&1
tail -2 "$OUT/abw_tests.log"
