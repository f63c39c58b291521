#!/bin/bash
# GPU-box: the overlapped KL loop (EK_KL_PIPE=1) against the standing one:
# swap-loop time and swap-log md5 on three graphs, then the KL parity tests
# under EK_KL_PIPE=1.  usage: tools/kl_pipe_check.sh TAG [pytest -k expr]
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
TAG="$1"; K="${2:-kl or swap or headline or results or cli or solve}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"; cd "$ROOT"
for v in 0 1; do
  echo "== EK_KL_PIPE=$v"
  EK_KL_PIPE=$v timeout -k 10 180 python3 tools/kl_ab.py 3 2>&1 | grep -v amdgpu.ids || exit $?
done > "$OUT/${TAG}_kl_ab.txt"
cat "$OUT/${TAG}_kl_ab.txt"
EK_KL_PIPE=1 timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "$K" \
  > "$OUT/${TAG}_tests.log" 2>&1
rc=$?
grep -E "FAIL|ERROR|passed|failed" "$OUT/${TAG}_tests.log" | tail -30
exit $rc
