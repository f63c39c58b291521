#!/bin/bash
# GPU box: PMC passes over the 10x resident solve (column-panel SpMV by
# default there): traffic, L2 hits, wave waits.  One pass per counter group.
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/panel_pmc"; mkdir -p "$OUT"; cd /tmp; export TMPDIR=/tmp
i=0
for ctr in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d "$OUT/p$i" -o p \
      -- python3 "$ROOT/tools/spmv_probe.py" resident ${1:-10.0} 10 > "$OUT/p$i.txt" 2>&1
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
for f in sorted(glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True)):
    agg = collections.defaultdict(list)
    for row in csv.DictReader(open(f)):
        if "spmv" in row["Kernel_Name"]:
            agg[(row["Kernel_Name"][:40], row["Counter_Name"])].append(float(row["Counter_Value"]))
    for (k, c), v in agg.items():
        print(f"{k:40s} {c:24s} n={len(v):4d} avg={sum(v)/len(v):.4g}")
PY
