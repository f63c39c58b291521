#!/bin/bash
# L2 and address-translation counters of the KL swap loop (through gpurun
# from the repo root): the counter names this gfx950 offers for the TCP /
# UTCL / TCC blocks, then one rocprofv3 --pmc pass per counter set given as
# arguments (quoted, space-separated) over tools/kl_ab.py.
# Output: gpurun_out/kl_pmc_cache/.
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/kl_pmc_cache"
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$OUT/list.txt" 2>&1 || true
grep -oE "\b(TCP|TCC|UTCL|TA|TD)_[A-Z0-9_]*(UTCL|TRANSLATION|TLB|HIT|MISS|TAG|PENDING|LATENCY)[A-Z0-9_]*" "$OUT/list.txt" | sort -u > "$OUT/names.txt" || true
i=0
for set in "$@"; do
    i=$((i + 1))
    # shellcheck disable=SC2086
    timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d "$OUT/p$i" -o kl -- python3 "$ROOT/tools/kl_ab.py" 1 > "$OUT/p$i.txt" 2>&1 || echo "pass $i failed: $set"
done
echo "pmc done"
