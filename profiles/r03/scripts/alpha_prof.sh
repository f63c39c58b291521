#!/bin/bash
# GPU box: kernel times of the headline file steps per alpha reduction:
# every projection workgroup re-reduces the SpMV's partials (default), the
# SpMV's last block does (EK_ALPHA_LAST=1), or the SpMV's blocks leave 256
# strided group sums (EK_ALPHA_GRP=1); then the Lanczos solves per variant.
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/alpha_prof"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for v in EK_ALPHA_GRP=0 EK_ALPHA_GRP=1 EK_ALPHA_LAST=1 EK_ALPHA_GRP=0 EK_ALPHA_GRP=1; do
  ( export $v; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$v" -o run \
      -- python3 "$ROOT/tools/spmv_probe.py" file 1.15lcc 1 1 3 > "$OUT/$v.txt" 2>&1 ) || exit 3
  echo "== $v"
  head -5 "$OUT/$v/run_kernel_stats.csv" | cut -d, -f1-4 | cut -c1-40,140-
done
cd "$ROOT"
timeout -k 10 300 python -u tools/restart_ab.py - EK_ALPHA_GRP=1 - EK_ALPHA_GRP=1 2>&1
