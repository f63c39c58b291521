cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 240 env EK_LANCZOS_TRACE=1 python3 -c "
import sys; sys.path.insert(0, 'tests'); from conftest import load_package
ek = load_package()
h = ek.Hypergraph.generate(1.15, 1).largest_component()[0]
c = ek.Context(0); c.spmv_setup_pins(h)
for _ in range(5): lam, v, st = c.lanczos_fiedler(); print(st['total_ms'], flush=True)
" > gpurun_out/restart_split.txt 2>&1
rc=$?
grep -E "factorization cycles|^[0-9]" gpurun_out/restart_split.txt
exit $rc
