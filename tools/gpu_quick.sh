#!/bin/bash
# Quick GPU iteration (through gpurun from the repo root): a subset of the -m gpu
# suite (pytest -k EXPR) and a short bench without the extra legs.
#   usage: tools/gpu_quick.sh TAG "pytest -k expression" [bench args...]
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
TAG="$1"; K="$2"; shift 2
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "$K" \
    > "$OUT/${TAG}_tests.log" 2>&1
rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed" "$OUT/${TAG}_tests.log" | tail -40
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc $rc: stopping"; exit $rc; fi
[ $rc -ne 0 ] && exit 1
timeout -k 10 600 python -u bench.py --no-extras "$@" > "$OUT/${TAG}_bench.json" 2> "$OUT/${TAG}_bench.err"
brc=$?
tail -5 "$OUT/${TAG}_bench.err"
python3 -c "
import json,sys; d=json.load(open('$OUT/${TAG}_bench.json'))
r=d['result']; print('value', d['value'], 'phases', r['phases_median_s']); print('resident', r['resident_solve'])
print('spmv us', d['roofline']['avg_launch_us'], 'frac', d['roofline']['frac'])"
exit $brc
