#!/usr/bin/env python3
"""Lab (not shipped): Lanczos matvec counts and lambda bits of the 1x synthetic
through the three setup paths (solve_file, host CSR, device build from the
pins), with and without the fp32 basis shadow.  usage: python tools/matvec_probe.py [MULT SEED]"""
import importlib.util
import os
import struct
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("ek", os.path.join(REPO, "eig-kl-algorithm_amd", "__init__.py"))
ek = importlib.util.module_from_spec(spec)
spec.loader.exec_module(ek)
mult = float(sys.argv[1]) if len(sys.argv) > 1 else 1.0
seed = int(sys.argv[2]) if len(sys.argv) > 2 else 1
h = ek.Hypergraph.generate(mult, seed)
work = tempfile.mkdtemp()
path = os.path.join(work, "g.hgr")
h.write(path)
ctx = ek.Context(0)
L = h.laplacian()
for b32 in (False, True):
    r, _ = ctx.solve_file(path, eig=1, out_dir=work, basis32=b32)
    print(f"b32={b32:d} solve_file       matvecs {r['lanczos']['matvecs']:5d} lambda {struct.pack('<d', r['lambda']).hex()}",
          flush=True)
    for name, setup in (("host csr", lambda: ctx.spmv_setup(h.nodes, 0, L.rowptr, L.col, L.val)),
                        ("pins", lambda: ctx.spmv_setup_pins(h))):
        setup()
        for rep in range(2):
            lam, v, st = ctx.lanczos_fiedler(basis32=b32)
            print(f"b32={b32:d} {name:9s} #{rep}  matvecs {st['matvecs']:5d} lambda {struct.pack('<d', lam).hex()} "
                  f"{st['total_ms']:.2f} ms", flush=True)
ctx.close()
