#!/bin/bash
# GPU box: HIP API + kernel trace (no counters) of one fresh gKL2 -EIG run on
# the headline workload: where the cold solve's extra time goes.
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/cold_trace"; mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 120 python -c "
import importlib.util,sys
spec=importlib.util.spec_from_file_location('ek','eig-kl-algorithm_amd/__init__.py'); ek=importlib.util.module_from_spec(spec); spec.loader.exec_module(ek)
ek.Hypergraph.generate(1.15,1).largest_component()[0].write('/tmp/h115.hgr')" || exit 1
mkdir -p /tmp/ekct && cd /tmp/ekct && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --stats --output-format csv -d "$OUT" -o ct \
    -- python3 "$ROOT/tools/cli_run.py" /tmp/h115.hgr -EIG --quiet > "$OUT/run.txt" 2>&1
