#!/bin/bash
# The headline SpMV's L2 behaviour inside the Lanczos solve against back to
# back, through gpurun from the repo root: kernel traces
# and one PMC pass each (TCC_HIT / TCC_MISS / TCC_EA0_RDREQ / _32B: the four
# TCC counters one pass holds) over
#   solve : tools/spmv_probe.py resident 1.15lcc 1 3   (3 resident solves)
#   b2b   : tools/spmv_probe.py b2b 1.15lcc 1 [fused]  (200 launches each)
# Output: gpurun_out/spmv_cache/<case>_{trace,pmc}/.
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/spmv_cache"
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
P="$ROOT/tools/spmv_probe.py"
run() {  # case, probe args...
    local c=$1; shift
    timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${c}_trace" -o p -- python3 "$P" "$@" > "$OUT/${c}_trace.txt" 2>&1
    timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --output-format csv -d "$OUT/${c}_pmc" -o p -- python3 "$P" "$@" > "$OUT/${c}_pmc.txt" 2>&1
}
run solve resident 1.15lcc 1 3
run b2b_plain b2b 1.15lcc 1
run b2b_fused b2b 1.15lcc 1 fused
echo "spmv cache lab done"
