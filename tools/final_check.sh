#!/bin/bash
# GPU-box: the full -m gpu suite + smoke() (tools/gpu_check.sh), then one
# bench run that keeps its rocprofv3 summaries (--prof-dir).
#   usage: tools/final_check.sh TAG
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
TAG="$1"
cd "$ROOT"
bash tools/gpu_check.sh "$TAG" "" nobench
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 900 python -u bench.py --prof-dir "gpurun_out/${TAG}_prof" > "gpurun_out/${TAG}_bench.json" 2> "gpurun_out/${TAG}_bench.err"
brc=$?
tail -c 1500 "gpurun_out/${TAG}_bench.json"
echo "pytest rc $rc bench rc $brc"
[ $rc -eq 0 ] && exit $brc
exit $rc
