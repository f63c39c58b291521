#!/bin/bash
# A/B of the parked WIP library (tools/build/wip) against the in-tree build
# (through gpurun from the repo root): KL loop time, Lanczos restarts A/B,
# 10x Lanczos, and the WIP's parity tests.
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out"
cd "$ROOT"
WIP="$ROOT/tools/build/wip/libeigkl_hip.so"
for v in main wip; do
  if [ $v = wip ]; then export EK_LIB_PATH=$WIP; else unset EK_LIB_PATH; fi
  timeout -k 10 200 python -u tools/kl_prof.py 1.15 > "$OUT/abw_klprof_$v.txt" 2>&1 || exit 3
  grep "prof=" "$OUT/abw_klprof_$v.txt" | sed "s/^/$v /"
  timeout -k 10 300 python -u tools/restart_ab.py - > "$OUT/abw_restart_$v.txt" 2>&1 || exit 4
  sed "s/^/$v /" "$OUT/abw_restart_$v.txt"
  REPS=1 timeout -k 10 200 python -u tools/lanczos_ab.py 10.0 - 2>&1 | sed "s/^/$v /" || exit 5
done
export EK_LIB_PATH=$WIP
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "kl or lcc or full_scale or solve or cli or lanczos or basis32 or panel" > "$OUT/abw_tests.log" 2>&1
tail -2 "$OUT/abw_tests.log"
