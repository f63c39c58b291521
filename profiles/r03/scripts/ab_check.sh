#!/bin/bash
# Lanczos mid-cycle check A/B on the GPU box: the lab under rocprofv3 kernel
# trace with check_every = each argument; idle gaps per solve.
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/ab_check"
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
for ce in "$@"; do
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d "$OUT/ce$ce" -o lab -- python3 "$ROOT/tools/lanczos_ab.py" 4 "$ce" > "$OUT/ce$ce.txt" 2>&1
  echo "== check_every $ce"; grep -E "syn1" "$OUT/ce$ce.txt"
  python3 "$ROOT/tools/gaps.py" "$OUT/ce$ce"
done
