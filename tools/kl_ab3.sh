#!/bin/bash
# KL A/B (tools/kl_ab2.sh) plus the stamped profile (tools/kl_prof.py) of each build
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
"$ROOT/tools/kl_ab2.sh" "$@" || exit 1
for b in "$@"; do
    echo "== prof $b"
    EK_LIB_PATH="$ROOT/eig-kl-algorithm_amd/$b/libeigkl_hip.so" timeout -k 10 200 python3 "$ROOT/tools/kl_prof.py" 2>&1 | grep -v amdgpu.ids || exit 1
done
