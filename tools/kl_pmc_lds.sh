#!/bin/bash
# LDS counters of the KL swap loop (one rocprofv3 --pmc pass over
# tools/kl_ab.py, its own kill limit).  Output: gpurun_out/kl_pmc_lds/.
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/kl_pmc_lds"
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES \
    --output-format csv -d "$OUT/p1" -o kl -- python3 "$ROOT/tools/kl_ab.py" 1 > "$OUT/p1.txt" 2>&1
echo "pmc done"
