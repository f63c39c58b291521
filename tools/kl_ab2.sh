#!/bin/bash
# KL swap-loop A/B of library builds on ONE GPU box: tools/kl_quick.py (the
# headline LCC, the 1x and 2x synthetics from their GPU splits; the swap-log
# md5 must not change) with each build in turn, twice (ABAB order).
#   usage: tools/kl_ab2.sh build_dir...   ("build" = the default build)
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
for pass in 1 2; do
  for b in "$@"; do
    echo "== $b (pass $pass)"
    EK_LIB_PATH="$ROOT/eig-kl-algorithm_amd/$b/libeigkl_hip.so" timeout -k 10 200 python3 "$ROOT/tools/kl_quick.py" 3 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
