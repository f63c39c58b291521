#!/bin/bash
# GPU box: the headline SpMV with a resident grid (EK_SPMV_PERSIST=k
# workgroups per CU) against the one-workgroup-per-row-block launch: rocprofv3
# kernel trace of the bench's file step (1 untimed + 3 solve_file steps) and
# 200 back-to-back fused launches, per k.   usage: tools/spmv_persist_lab.sh [k ...]
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd /tmp && export TMPDIR=/tmp
OUT="$ROOT/gpurun_out/persist"
mkdir -p "$OUT"
for k in ${@:-0 1 2 4 8}; do
    EK_SPMV_PERSIST=$k timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/k$k" -o p -- \
        python3 "$ROOT/tools/spmv_probe.py" file 1.15lcc 1 1 3 > "$OUT/k$k.log" 2>&1 || { echo "k=$k failed"; exit 1; }
    echo "== k=$k" >> "$OUT/summary.txt"
    python3 "$ROOT/tools/kstats.py" "$OUT/k$k" 8 >> "$OUT/summary.txt"
    EK_SPMV_PERSIST=$k timeout -k 10 120 python3 "$ROOT/tools/spmv_probe.py" b2b 1.15lcc 1 solve >> "$OUT/summary.txt" 2>&1 || exit 1
    EK_SPMV_PERSIST=$k timeout -k 10 120 python3 "$ROOT/tools/spmv_probe.py" b2b 1.15lcc 1 >> "$OUT/summary.txt" 2>&1 || exit 1
done
grep -E "== k|spmv_adaptive|probe" "$OUT/summary.txt"
