#!/bin/bash
# Build an A/B variant of libeigkl_hip.so from a git revision's sources into
# eig-kl-algorithm_amd/build_<name>/ (git-ignored; travels to the GPU box;
# load it with EK_LIB_PATH).  usage: tools/ab_build.sh NAME REV [make vars...]
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
NAME="$1"; REV="$2"; shift 2
SRC="/tmp/ab_src_$NAME"
rm -rf "$SRC" && mkdir -p "$SRC/pkg/csrc" "$SRC/include"
if [ "$REV" = WORK ]; then  # the working tree as it is
    mkdir -p "$SRC/eig-kl-algorithm_amd" && cp -r "$ROOT/eig-kl-algorithm_amd/csrc" "$SRC/eig-kl-algorithm_amd/" && cp -r "$ROOT/include" "$SRC/"
else
    git -C "$ROOT" archive "$REV" eig-kl-algorithm_amd/csrc include | tar -x -C "$SRC"
fi
cp "$SRC"/eig-kl-algorithm_amd/csrc/* "$SRC/pkg/csrc/"

cp "$ROOT/eig-kl-algorithm_amd/Makefile" "$SRC/pkg/"
make -C "$SRC/pkg" -j8 OUT="$ROOT/eig-kl-algorithm_amd/build_$NAME" "$@" "$ROOT/eig-kl-algorithm_amd/build_$NAME/libeigkl_hip.so" >/dev/null
echo "built eig-kl-algorithm_amd/build_$NAME/libeigkl_hip.so from $REV"
