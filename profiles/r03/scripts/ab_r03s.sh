#!/bin/bash
# Round-3 fp32-shadow update / alpha placement A/B (through gpurun from the repo root)
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
TAG="${1:-r03t}"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT/$TAG"
cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "lanczos" \
    > "$OUT/${TAG}_tests.log" 2>&1
rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed" "$OUT/${TAG}_tests.log" | tail -60
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
REPS=2 timeout -k 10 300 python -u tools/lanczos_ab.py 1.0,10.0 - EK_BASIS32=0 EK_ALPHA_LAST=0 EK_BASIS32=0,EK_ALPHA_LAST=0 \
    > "$OUT/${TAG}_ab.txt" 2>&1 || exit $?
cat "$OUT/${TAG}_ab.txt"
cd /tmp; export TMPDIR=/tmp
for v in base a0; do
  if [ $v = a0 ]; then export EK_ALPHA_LAST=0; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$TAG/$v" -o "$v" \
    -- python3 "$ROOT/tools/lanczos_ab.py" 1.0 - > "$OUT/$TAG/${v}.txt" 2>&1 || exit $?
done
echo ab done
