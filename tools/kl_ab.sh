#!/bin/bash
# KL swap-loop A/B of library builds on the GPU box (through gpurun from the
# repo root): tools/kl_ab.py with each build, in turn, twice (ABAB order).
#   usage: tools/kl_ab.sh build_dir...
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
for pass in 1 2; do
  for b in "$@"; do
    n=$(basename "$b")
    echo "== $n (pass $pass)"
    EK_LIB_PATH="$ROOT/eig-kl-algorithm_amd/$n/libeigkl_hip.so" timeout -k 10 150 python3 "$ROOT/tools/kl_ab.py" 5 2>&1 | grep -v amdgpu.ids
  done
done
