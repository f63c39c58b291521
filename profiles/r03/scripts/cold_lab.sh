#!/bin/bash
# GPU box: the fresh-process wall of gKL2 -EIG split by start-up event, on the
# headline workload (largest component of the 1.15x seed-1 synthetic), with
# runtime variants, alternated so that box drift shows.
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 120 python -c "
import importlib.util,sys
spec=importlib.util.spec_from_file_location('ek','eig-kl-algorithm_amd/__init__.py'); ek=importlib.util.module_from_spec(spec); spec.loader.exec_module(ek)
ek.Hypergraph.generate(1.15,1).largest_component()[0].write('/tmp/h115.hgr')" || exit 1
for v in ${VARIANTS:-EK_PRELOAD=0 EK_PRELOAD=1 EK_PRELOAD=0 EK_PRELOAD=1}; do
  echo "== variant [$v]"
  timeout -k 10 300 python tools/cold_probe.py /tmp/h115.hgr 5 $v || exit 2
done
