#!/bin/bash
# LDS / SQ counters of the two KL swap loops (EK_KL_PIPE=0 / 1), one rocprofv3
# --pmc pass each over tools/kl_ab.py, per swap-loop dispatch.
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/kl_pipe_pmc"; mkdir -p "$OUT"
cd /tmp; export TMPDIR=/tmp
for v in 0 1; do
  EK_KL_PIPE=$v timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU \
    --output-format csv -d "$OUT/p$v" -o kl -- python3 "$ROOT/tools/kl_ab.py" 1 > "$OUT/p$v.txt" 2>&1 || exit 1
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
for v in (0, 1):
    f = glob.glob(f"{out}/p{v}/**/*counter_collection.csv", recursive=True)[0]
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        if "swap" not in r["Kernel_Name"]: continue
        agg[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    print(f"EK_KL_PIPE={v}:", open(f"{out}/p{v}.txt").read().strip().replace("\n", " | "))
    for d, c in sorted(agg.items(), key=lambda x: int(x[0])):
        print("  dispatch", d, {k: int(x) for k, x in sorted(c.items())})
PY
