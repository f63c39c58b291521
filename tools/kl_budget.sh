#!/bin/bash
# The KL swap loop's cycle budget on the headline workload (VERDICT r3
# next-7), through gpurun from the repo root:
#   1. tools/kl_prof.py: plain / EK_KL_PROF=1 phase stamps and per-wave
#      timelines / plain again (us/swap);
#   2. two rocprofv3 --pmc passes of SQ counters over the same script (8 SQ
#      counters a pass; the plain k_kl_swap_loop<false, ...> dispatches are
#      the ones to read).
# Output: gpurun_out/kl_budget/.
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/${KL_BUDGET_DIR:-kl_budget}"
mkdir -p "$OUT"
timeout -k 10 120 python3 "$ROOT/tools/kl_prof.py" > "$OUT/prof.txt" 2>&1
cd /tmp
export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU \
    --output-format csv -d "$OUT/p1" -o kl -- python3 "$ROOT/tools/kl_prof.py" > "$OUT/p1.txt" 2>&1
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS \
    --output-format csv -d "$OUT/p2" -o kl -- python3 "$ROOT/tools/kl_prof.py" > "$OUT/p2.txt" 2>&1
echo "kl budget done"
