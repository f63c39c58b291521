#!/bin/bash
# Lab (run through gpurun): process wall and phase log of the drop-in gKL2 -EIG
# on the ibm18-shape synthetic written to a .hgr file.
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
W=$(mktemp -d)
cd "$W"
python3 - "$ROOT" <<'PY'
import importlib.util, os, sys
spec = importlib.util.spec_from_file_location("eigkl_amd", os.path.join(sys.argv[1], "eig-kl-algorithm_amd", "__init__.py"))
ek = importlib.util.module_from_spec(spec); spec.loader.exec_module(ek)
ek.Hypergraph.generate(1.0, 1).write("ibm18_shape.hgr")
PY
T="$ROOT/eig-kl-algorithm_amd/build/bin/gKL2"
for i in 1 2 3; do
    s=$EPOCHREALTIME
    timeout -k 10 60 "$T" ibm18_shape.hgr -EIG > "out_$i.txt"
    e=$EPOCHREALTIME
    awk -v a="$s" -v b="$e" -v i="$i" 'BEGIN { printf "run %d wall %.3f s\n", i, b - a }'
done
tail -30 out_3.txt
