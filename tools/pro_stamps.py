#!/usr/bin/env python3
"""Lab: where the time of the projection launch with the in-launch decision
goes.  Needs a build with -DEK_PRO_STAMPS (tools/ab_build.sh stamps WORK
EXTRA_DEFS=-DEK_PRO_STAMPS) loaded through EK_LIB_PATH.  Runs resident
headline solves, reads the per-workgroup stamps (kernels_lanczos.hip
g_pro_stamps: role, entry, two phase marks, exit, decision; 100 MHz clock)
of steps 20..99 of the last cycle to reach them, and prints, per step kind
(skipped / projecting), the medians over steps of: the decider's publish
time, the column-group-0 workgroups' f' and norm hand-off, the pollers' and
the update's decision times and the last exit, all relative to the first
workgroup's entry.  usage: python tools/pro_stamps.py [MULT[lcc] SEED]"""
import ctypes
import importlib.util
import os
import statistics
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("eigkl_amd", os.path.join(REPO, "eig-kl-algorithm_amd", "__init__.py"))
ek = importlib.util.module_from_spec(spec)
spec.loader.exec_module(ek)
LO, NS, WG, W = 20, 80, 2048, 6
ROLES = {1: "decider", 2: "decider-slot", 3: "cg0", 4: "cg>0", 5: "update"}

if sys.argv[1:2] == ["--from"]:
    S = np.load(sys.argv[2])
else:
    a, sd = (sys.argv[1:3] + ["1.15lcc", "1"][len(sys.argv[1:3]):])[:2]
    lcc = a.endswith("lcc")
    h = ek.Hypergraph.generate(float(a[:-3] if lcc else a), int(sd))
    if lcc:
        h, _ = h.largest_component()
    c = ek.Context(0)
    c.spmv_setup_pins(h)
    for _ in range(2):
        lam, v, st = c.lanczos_fiedler()
    print({k: st[k] for k in ("matvecs", "restarts", "projected_steps", "total_ms")}, flush=True)
    fn = ek._lib.ek_lab_pro_stamps
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_longlong]
    buf = np.zeros(NS * WG * W, dtype=np.uint64)
    assert fn(buf.ctypes.data, buf.size) == buf.size
    c.close()
    S = buf.reshape(NS, WG, W).astype(np.int64)
if os.environ.get("EK_STAMPS_OUT"):  # the raw table, for offline looks (tools/pro_stamps.py --from FILE)
    np.save(os.environ["EK_STAMPS_OUT"], S)

rows = {1: [], 2: []}
for k in range(NS):
    s = S[k]
    live = s[:, 0] > 0
    if not live.any():
        continue
    nwg = int(np.nonzero(live)[0].max()) + 1
    s = s[:nwg]
    dec = int(s[0, 5])
    if dec not in (1, 2):
        continue
    t0 = s[:, 1].min()
    rel = lambda x: (x - t0) / 100.0  # us

    def role(r):
        return s[s[:, 0] == r]
    d = role(1)
    cg0, cgx, up = role(3), role(4), role(5)
    r = {"step": LO + k, "nwg": nwg,
         "dispatch_span": rel(s[:, 1].max()),
         "decider_entry": rel(d[0, 1]), "decider_publish": rel(d[0, 2]),
         "cg0_entry_med": rel(np.median(cg0[:, 1])), "cg0_fprime_med": rel(np.median(cg0[:, 2])),
         "cg0_entry_max": rel(cg0[:, 1].max()), "cg0_fprime_p90": rel(np.percentile(cg0[:, 2], 90)),
         "cg0_fprime_max": rel(cg0[:, 2].max()),
         "cg0_tail_nonlast_med": float(np.median(np.sort(cg0[:, 3] - cg0[:, 2])[:-1])) / 100.0,
         "cg0_norm_handoff_max": rel(cg0[:, 3].max()),
         "cgx_seen_med": rel(np.median(cgx[:, 2])) if len(cgx) else 0.0,
         "upd_entry_med": rel(np.median(up[:, 1])) if len(up) else 0.0,
         "upd_seen_med": rel(np.median(up[:, 2])) if len(up) else 0.0,
         "upd0_norm_in": rel(up[0, 3]) if len(up) and up[0, 3] > 0 else 0.0,
         "last_exit": rel(s[:, 4].max()),
         "cg0_exit_max": rel(cg0[:, 4].max()), "cgx_exit_max": rel(cgx[:, 4].max()) if len(cgx) else 0.0,
         "upd_exit_max": rel(up[:, 4].max()) if len(up) else 0.0}
    rows[dec].append(r)

for dec, name in ((1, "skipped"), (2, "projecting")):
    rs = rows[dec]
    print(f"== {name} steps: {len(rs)}")
    if not rs:
        continue
    for key in rs[0]:
        if key == "step":
            continue
        vals = [r[key] for r in rs]
        print(f"  {key:22s} median {statistics.median(vals):8.2f}  min {min(vals):8.2f}  max {max(vals):8.2f}")
    r = rs[len(rs) // 2]
    print(f"  example step {r['step']}: " + ", ".join(f"{k}={v:.2f}" for k, v in r.items() if k != "step"))
