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
4. ``--seeded``: runs ``oracle/_ref/cKL_seeded`` (the same reference source,
   its std::random_device seed taken from $EK_REF_SEED: oracle/ref_seed.h) as
   ``cKL <c>.hgr`` (random init, cKL.cpp:176-192) for the (circuit, seed)
   pairs in SEEDED and keeps ``results/<c>.hgr_KL_CutSize_output.txt`` as
   ``tests/golden/ref_results_seed/<c>.seed<S>.txt``.
5. ``--lcc [MULT]``: the largest connected component of the product
   generator's MULT x (default 1.0) seed-1 synthetic (ek_hgr_largest_component;
   1.0x: 184,306 nodes; 1.15x: 211,813, the bench's headline workload), its
   Fiedler split from the oracle Lanczos (median split, sign: largest |v|
   positive), and the REAL reference cKL run on it (``cKL <name>.hgr -EIG``,
   ~40 min on 4 cores at 1.0x): ``tests/golden/<name>/`` (syn1_lcc,
   syn115_lcc) keeps the packed split bits, lambda / median / the near-median
   nodes, and the gzipped reference results file.

Usage: python oracle/gen_golden.py [circuit ...]   (default: all four)
       python oracle/gen_golden.py --seeded
       python oracle/gen_golden.py --lcc [MULT [EIG_FILE REF_RESULTS_FILE]]
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


SEEDED = [("fract", 1), ("fract", 7), ("fract", 12345), ("ibm01", 1)]


def seeded():
    exe = os.path.join(HERE, "_ref", "cKL_seeded")
    if not os.path.exists(exe):
        subprocess.check_call(["make", "-f", os.path.join(HERE, "ref.mk")])
    dst = os.path.join(GOLD, "ref_results_seed")
    os.makedirs(dst, exist_ok=True)
    runs_path = os.path.join(GOLD, "ref_runs.json")
    runs = json.load(open(runs_path)) if os.path.exists(runs_path) else {}
    for c, seed in SEEDED:
        hgr = f"{c}.hgr"
        with tempfile.TemporaryDirectory() as tmp:
            shutil.copy(os.path.join(REF, "circuit", hgr), os.path.join(tmp, hgr))
            t0 = time.time()
            subprocess.run([exe, hgr], cwd=tmp, capture_output=True, text=True, check=True,
                           env=dict(os.environ, EK_REF_SEED=str(seed)))
            runs[f"{c}.seed{seed}"] = {"wall_s": round(time.time() - t0, 3), "threads": os.cpu_count(),
                                       "binary": "oracle/_ref/cKL_seeded"}
            shutil.copy(os.path.join(tmp, "results", f"{hgr}_KL_CutSize_output.txt"),
                        os.path.join(dst, f"{c}.seed{seed}.txt"))
        print(c, seed, runs[f"{c}.seed{seed}"], flush=True)
    json.dump(runs, open(runs_path, "w"), indent=1, sort_keys=True)


def lcc_name(mult):
    return "syn1_lcc" if mult == 1.0 else "syn%s_lcc" % f"{mult:g}".replace(".", "")


def lcc(mult="1.0", eig_file=None, ref_results=None):
    """syn1_lcc / syn115_lcc fixture.  eig_file / ref_results: an EIG file
    written for the component and the reference results of a cKL run on it
    (the run takes ~40 min on 4 cores), else both are made here (oracle
    Lanczos on all host cores, then the reference)."""
    import gzip
    import numpy as np
    sys.path.insert(0, os.path.join(REPO, "tests"))
    sys.path.insert(0, HERE)
    from conftest import load_package
    import oracle
    ek = load_package()
    mult = float(mult)
    name = lcc_name(mult)
    dst = os.path.join(GOLD, name)
    os.makedirs(dst, exist_ok=True)
    h, _ = ek.Hypergraph.generate(mult, 1).largest_component()
    with tempfile.TemporaryDirectory() as tmp:
        path = os.path.join(tmp, f"{name}.hgr")
        h.write(path)
        meta = {"nodes": h.nodes, "nets": h.nets, "generator": {"mult": mult, "seed": 1},
                "made_by": f"oracle/gen_golden.py --lcc {mult:g}: oracle Lanczos (sign: largest |v| positive), "
                           f"median split, real reference cKL {name}.hgr -EIG"}
        if eig_file is None:
            g = oracle.Graph.read(path)
            oracle.set_threads(os.cpu_count())
            lam, v, st = g.lanczos(deflate=True)
            v = v * np.sign(v[np.argmax(np.abs(v))])
            med, bits = ek.median_split(v)
            meta.update(oracle_matvecs=st["matvecs"], oracle_residual=st["residual"])
            os.makedirs(os.path.join(tmp, "pre_saved_EIG"))
            eig_file = os.path.join(tmp, "pre_saved_EIG", f"{name}.hgr_out.txt")
            ek.eig_write(eig_file, lam, med, bits, v)
        lam, med, bits, v, _, _ = ek.eig_read(eig_file, h.nodes)
        near = np.flatnonzero(np.abs(v - med) <= 1e-8)
        meta.update(lambda1=lam, median=med, near_median_nodes=near.tolist())
        np.save(os.path.join(dst, "split_bits.npy"), np.packbits(bits))
        if ref_results is None:
            os.makedirs(os.path.join(tmp, "pre_saved_EIG"), exist_ok=True)
            if os.path.abspath(eig_file) != os.path.join(tmp, "pre_saved_EIG", f"{name}.hgr_out.txt"):
                shutil.copy(eig_file, os.path.join(tmp, "pre_saved_EIG", f"{name}.hgr_out.txt"))
            t0 = time.time()
            r = subprocess.run([CKL, f"{name}.hgr", "-EIG"], cwd=tmp, capture_output=True, text=True, check=True)
            meta["reference_wall_s"] = round(time.time() - t0, 1)
            meta["reference_summary"] = [ln.strip() for ln in r.stdout.splitlines() if ":" in ln and (
                "Total iterations" in ln or "Initial cut" in ln or "Best cut" in ln or "Number of cores" in ln)]
            ref_results = os.path.join(tmp, "results", f"{name}.hgr_KL_CutSize_EIG_output.txt")
            val = lambda key: [ln.split(":", 1)[1].strip() for ln in meta["reference_summary"] if ln.startswith(key)][0]
            meta["reference_run"] = {"binary": "oracle/_ref/cKL (built by oracle/ref.mk from /root/reference/cKL.cpp)",
                                     "cmd": f"cKL {name}.hgr -EIG", "process_wall_s": meta["reference_wall_s"],
                                     "iterations": int(val("Total iterations")),
                                     "initial_cut": val("Initial cut size"), "best_cut": val("Best cut size achieved")}
        if os.path.exists(ref_results):
            with open(ref_results, "rb") as f, gzip.open(os.path.join(dst, "ref_results.txt.gz"), "wb", 9) as z:
                z.write(f.read())
        json.dump(meta, open(os.path.join(dst, "meta.json"), "w"), indent=1)
        print(name, {k: meta[k] for k in ("nodes", "lambda1", "median")}, len(near), "near-median", flush=True)


def main(argv):
    if len(argv) > 1 and argv[1] == "--seeded":
        return seeded()
    if len(argv) > 1 and argv[1] == "--lcc":
        return lcc(*argv[2:5])
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
