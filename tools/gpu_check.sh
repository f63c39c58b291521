#!/bin/bash
# GPU-box check (run through gpurun from the repo root): the -m gpu suite,
# smoke(), then one bench run.  Every GPU step has its own time limit; a
# test-assertion failure (pytest rc 1) still lets the bench run, anything
# else (fault, abort, timeout) ends the script there.
#   usage: tools/gpu_check.sh TAG [pytest -k expression]
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
TAG="${1:-r02}"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
cd "$ROOT"
K=()
[ -n "$2" ] && K=(-k "$2")
timeout -k 10 1200 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread "${K[@]}" \
    > "$OUT/${TAG}_gpu_tests.log" 2>&1
rc=$?
tail -5 "$OUT/${TAG}_gpu_tests.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc $rc: stopping"; exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/${TAG}_smoke.log" 2>&1 || { echo "smoke failed"; cat "$OUT/${TAG}_smoke.log" | tail -20; exit 3; }
tail -2 "$OUT/${TAG}_smoke.log"
[ "$3" = "nobench" ] && exit $rc
timeout -k 10 900 python -u bench.py > "$OUT/${TAG}_bench.json" 2> "$OUT/${TAG}_bench.err"
brc=$?
tail -c 3000 "$OUT/${TAG}_bench.json"
tail -20 "$OUT/${TAG}_bench.err"
echo "pytest rc $rc bench rc $brc"
exit $brc
