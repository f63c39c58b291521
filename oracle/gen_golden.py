#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/ (test infrastructure only).

Runs in THIS container (the only place /root/reference exists):

1. Copies the reference's shipped DATA files (inputs and reference outputs, no
   source): ``circuit/*.hgr`` and ``pre_saved_EIG/*.hgr_out.txt`` (the cEIG
   golden Fiedler files) into ``tests/golden/circuit`` and
   ``tests/golden/pre_saved_EIG``.
2. Runs the REAL reference cKL (built by ``make -f oracle/ref.mk`` into
   ``oracle/_ref/cKL`` from /root/reference/cKL.cpp) as ``cKL <c>.hgr -EIG`` in
   a scratch working directory, exactly as the reference README runs it, and
   copies its ``results/<c>.hgr_KL_CutSize_EIG_output.txt`` (cKL.cpp:315,380)
   to ``tests/golden/ref_results/``.  These rows (iteration, fp32 cut, fp32
   gain at 6 significant digits) pin the oracle restatement and the HIP path.
3. Records wall time / thread count per run in ``tests/golden/ref_runs.json``.

Usage: python oracle/gen_golden.py [circuit ...]   (default: all four)
"""
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

REF = os.environ.get("EK_REFERENCE", "/root/reference")
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
GOLD = os.path.join(REPO, "tests", "golden")
CKL = os.path.join(HERE, "_ref", "cKL")
CIRCUITS = ["fract", "ibm01", "industry2", "ibm10"]


def main(argv):
    names = argv[1:] or CIRCUITS
    if not os.path.exists(CKL):
        subprocess.check_call(["make", "-f", os.path.join(HERE, "ref.mk")])
    for sub in ("circuit", "pre_saved_EIG", "ref_results"):
        os.makedirs(os.path.join(GOLD, sub), exist_ok=True)
    runs_path = os.path.join(GOLD, "ref_runs.json")
    runs = json.load(open(runs_path)) if os.path.exists(runs_path) else {}
    for c in names:
        hgr = f"{c}.hgr"
        eig = f"{c}.hgr_out.txt"
        shutil.copy(os.path.join(REF, "circuit", hgr), os.path.join(GOLD, "circuit", hgr))
        shutil.copy(os.path.join(REF, "pre_saved_EIG", eig), os.path.join(GOLD, "pre_saved_EIG", eig))
        with tempfile.TemporaryDirectory() as tmp:
            os.makedirs(os.path.join(tmp, "circuit"))
            os.makedirs(os.path.join(tmp, "pre_saved_EIG"))
            shutil.copy(os.path.join(REF, "circuit", hgr), os.path.join(tmp, "circuit", hgr))
            shutil.copy(os.path.join(REF, "pre_saved_EIG", eig), os.path.join(tmp, "pre_saved_EIG", eig))
            t0 = time.time()
            out = subprocess.run([CKL, os.path.join("circuit", hgr), "-EIG"], cwd=tmp,
                                 capture_output=True, text=True, check=True).stdout
            wall = time.time() - t0
            res = f"{hgr}_KL_CutSize_EIG_output.txt"
            shutil.copy(os.path.join(tmp, "results", res), os.path.join(GOLD, "ref_results", res))
        summary = [ln.strip() for ln in out.splitlines() if ":" in ln and (
            "Total iterations" in ln or "Initial cut" in ln or "Best cut" in ln or "Number of cores" in ln)]
        runs[c] = {"wall_s": round(wall, 3), "threads": os.cpu_count(), "summary": summary}
        print(c, runs[c], flush=True)
    json.dump(runs, open(runs_path, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main(sys.argv)
