#!/usr/bin/env python3
"""Lab: the KL adjacency host build (ek_kl_graph_build) on the headline workload; EK_TRACE=1 prints its phases."""
import sys, time
sys.path.insert(0, "tests")
from conftest import load_package
ek = load_package()
h = ek.Hypergraph.generate(1.15, 1).largest_component()[0]
for _ in range(4):
    t = time.perf_counter(); G = h.kl_graph(); print("kl_graph %.2f ms" % ((time.perf_counter() - t) * 1e3), flush=True)
