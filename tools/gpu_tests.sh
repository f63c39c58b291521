#!/bin/bash
# GPU-box: a subset of the -m gpu suite (pytest -k / file args), own time limit.
#   usage: tools/gpu_tests.sh TAG [pytest args...]
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
TAG="$1"; shift
mkdir -p "$ROOT/gpurun_out"
cd "$ROOT"
timeout -k 10 900 python -u -m pytest -m gpu -v --timeout 600 --timeout-method thread "$@" \
    > "gpurun_out/${TAG}_gpu_tests.log" 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" "gpurun_out/${TAG}_gpu_tests.log" | tail -40
exit $rc
