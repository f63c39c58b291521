#!/bin/bash
# A/B of library builds on the GPU box (through gpurun from the repo root):
# for each build dir given, the Lanczos lab under rocprofv3 kernel-trace
# stats.  Each GPU step has its own limit; stop at the first failure.
#   usage: tools/ab_lab.sh TAG build_dir...
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
TAG="$1"; shift
OUT="$ROOT/gpurun_out/ab_$TAG"
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
for b in "$@"; do
  n=$(basename "$b")
  EK_LIB_PATH="$ROOT/eig-kl-algorithm_amd/$n/libeigkl_hip.so" timeout -k 10 240 rocprofv3 --kernel-trace --stats \
      --output-format csv -d "$OUT/$n" -o lab -- python3 "$ROOT/tools/lanczos_ab.py" 6 > "$OUT/$n.txt" 2>&1
  cat "$OUT/$n.txt" | grep -v amdgpu.ids
  python3 "$ROOT/tools/kstats.py" "$OUT/$n" 12
done
