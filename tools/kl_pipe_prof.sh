#!/bin/bash
# GPU-box: the overlapped KL loop's stamped profile (EK_KL_PROF) and its
# swap-loop time against the standing loop.  usage: tools/kl_pipe_prof.sh TAG
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
TAG="$1"; OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"; cd "$ROOT"
{
  EK_KL_PIPE=1 EK_KL_PROF=1 timeout -k 10 120 python3 tools/kl_ab.py 1 2>&1 || exit 1
  for v in 0 1; do
    echo "== EK_KL_PIPE=$v"
    EK_KL_PIPE=$v timeout -k 10 180 python3 tools/kl_ab.py 3 2>&1 || exit 1
  done
} | grep -v amdgpu.ids > "$OUT/${TAG}_kl_pipe.txt"
rc=${PIPESTATUS[0]}
cat "$OUT/${TAG}_kl_pipe.txt"
exit $rc
