#!/bin/bash
# GPU box: restart A/B of the parked build (tools/build/wip) against the
# in-tree one (restart_ab + the factorization/restart split of lanczos_trace).
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"; cd "$ROOT"
for v in new old; do
  if [ $v = old ]; then export EK_LIB_PATH="$ROOT/tools/build/wip/libeigkl_hip.so"; else unset EK_LIB_PATH; fi
  timeout -k 10 300 python -u tools/restart_ab.py - > "$OUT/abq_restart_$v.txt" 2>&1 || exit 4
  sed "s/^/$v /" "$OUT/abq_restart_$v.txt"
  EK_LANCZOS_TRACE=1 timeout -k 10 100 python -u tools/lanczos_trace.py > "$OUT/abq_trace_$v.txt" 2>&1 || exit 5
  grep factorization "$OUT/abq_trace_$v.txt" | sed "s/^/$v /"
done
