#!/bin/bash
# GPU box: the fresh-process wall of gKL2 -EIG split by start-up event, on the
# 1x synthetic (the bench workload) and ibm01, with a few runtime variants.
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 120 python -c "
import importlib.util,sys
spec=importlib.util.spec_from_file_location('ek','eig-kl-algorithm_amd/__init__.py'); ek=importlib.util.module_from_spec(spec); spec.loader.exec_module(ek)
ek.Hypergraph.generate(1.0,1).write('/tmp/syn1.hgr')" || exit 1
for v in "" "EK_THREADS=1" "EK_FAST_EXIT=1" "EK_FAST_EXIT=1 EK_NO_DESTROY=1" "" ; do
  echo "== variant [$v]"
  timeout -k 10 300 python tools/cold_probe.py /tmp/syn1.hgr 5 $v || exit 2
done
