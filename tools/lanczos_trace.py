"""Lab (not shipped): the Lanczos restart history (EK_LANCZOS_TRACE=1 lines on
stderr) on the shipped circuits and the 1x synthetic and its largest
component.  usage: EK_LANCZOS_TRACE=1 python tools/lanczos_trace.py"""
import importlib.util
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("eigkl_amd", os.path.join(REPO, "eig-kl-algorithm_amd", "__init__.py"))
ek = importlib.util.module_from_spec(spec)
spec.loader.exec_module(ek)
ctx = ek.Context(0)
h1 = ek.Hypergraph.generate(1.0, 1)
cases = [(c, ek.Hypergraph.read(os.path.join(REPO, "tests", "golden", "circuit", f"{c}.hgr")))
         for c in ("ibm01", "industry2", "ibm10")]
cases += [("syn1", h1), ("syn1_lcc", h1.largest_component()[0])]
for name, h in cases:
    L = h.laplacian()
    ctx.spmv_setup(h.nodes, 0, L.rowptr, L.col, L.val)
    print(f"=== {name} n={h.nodes}", file=sys.stderr, flush=True)
    lam, v, st = ctx.lanczos_fiedler()
    print(f"=== {name}: lambda {lam!r} matvecs {st['matvecs']} restarts {st['restarts']} residual {st['residual']:.3e}",
          file=sys.stderr, flush=True)
ctx.close()
