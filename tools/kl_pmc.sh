#!/bin/bash
# SQ counters of the KL swap loop (through gpurun from the repo root): two
# separate rocprofv3 --pmc passes over tools/kl_ab.py (one run per dataset),
# each under its own kill limit.  Output: gpurun_out/kl_pmc/<pass>/.
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/kl_pmc"
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS \
    --output-format csv -d "$OUT/p1" -o kl -- python3 "$ROOT/tools/kl_ab.py" 1 > "$OUT/p1.txt" 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VMEM SQ_ACTIVE_INST_MISC \
    --output-format csv -d "$OUT/p2" -o kl -- python3 "$ROOT/tools/kl_ab.py" 1 > "$OUT/p2.txt" 2>&1
echo "pmc done"
