#!/bin/bash
# GPU box: the headline SpMV per library build and env setting, on ONE box:
# rocprofv3 kernel trace of the bench's file step (1 untimed + 3 solve_file
# steps), and 200 back-to-back launches (fused as the solve, and plain).
#   usage: tools/spmv_ab.sh TAG "label|build_dir|ENV=V ..." ...
#   (build_dir "." = eig-kl-algorithm_amd/build; WL=... overrides the workload)
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
TAG="$1"; shift
WL="${WL:-1.15lcc 1}"
cd /tmp && export TMPDIR=/tmp
OUT="$ROOT/gpurun_out/spmv_ab_$TAG"
mkdir -p "$OUT"
for spec in "$@"; do
    IFS='|' read -r label bdir envs <<< "$spec"
    lib="$ROOT/eig-kl-algorithm_amd/${bdir/#./build}/libeigkl_hip.so"
    [ "$bdir" = "." ] && lib="$ROOT/eig-kl-algorithm_amd/build/libeigkl_hip.so"
    echo "== $label ($bdir $envs)" >> "$OUT/summary.txt"
    env EK_LIB_PATH="$lib" $envs timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$label" -o p -- \
        python3 "$ROOT/tools/spmv_probe.py" file $WL 1 3 > "$OUT/$label.log" 2>&1 || { echo "$label failed"; tail -5 "$OUT/$label.log"; exit 1; }
    python3 "$ROOT/tools/kstats.py" "$OUT/$label" 6 >> "$OUT/summary.txt"
    env EK_LIB_PATH="$lib" $envs timeout -k 10 120 python3 "$ROOT/tools/spmv_probe.py" b2b $WL solve >> "$OUT/summary.txt" 2>&1 || exit 1
    env EK_LIB_PATH="$lib" $envs timeout -k 10 120 python3 "$ROOT/tools/spmv_probe.py" b2b $WL >> "$OUT/summary.txt" 2>&1 || exit 1
done
grep -E "^==|spmv|probe|gemvt|kl_swap" "$OUT/summary.txt"
