#!/bin/bash
# GPU box: the 10x column-panel SpMV per library build (A/B): rocprofv3 kernel
# trace of one resident 10x Lanczos solve, and 200 back-to-back launches.
#   usage: tools/panel_ab.sh TAG build_dir...   ("build" = the default build)
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
TAG="$1"; shift
cd /tmp && export TMPDIR=/tmp
OUT="$ROOT/gpurun_out/panel_ab_$TAG"
mkdir -p "$OUT"
for b in "$@"; do
    lib="$ROOT/eig-kl-algorithm_amd/$b/libeigkl_hip.so"
    echo "== $b" >> "$OUT/summary.txt"
    EK_LIB_PATH="$lib" timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$b" -o p -- \
        python3 "$ROOT/tools/spmv_probe.py" resident 10 10 > "$OUT/$b.log" 2>&1 || { echo "$b failed"; tail -5 "$OUT/$b.log"; exit 1; }
    python3 "$ROOT/tools/kstats.py" "$OUT/$b" 5 >> "$OUT/summary.txt"
    EK_LIB_PATH="$lib" timeout -k 10 120 python3 "$ROOT/tools/spmv_probe.py" b2b 10 10 solve >> "$OUT/summary.txt" 2>&1 || exit 1
done
grep -E "^==|panel|probe" "$OUT/summary.txt"
