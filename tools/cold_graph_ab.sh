# GPU box: fresh-process wall of gKL2 -EIG on the headline with the Lanczos
# chunk graphs (default) and without (EK_LANCZOS_GRAPH=0), alternating.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 python3 -c "
import importlib.util
spec=importlib.util.spec_from_file_location('ek','eig-kl-algorithm_amd/__init__.py'); ek=importlib.util.module_from_spec(spec); spec.loader.exec_module(ek)
ek.Hypergraph.generate(1.15,1).largest_component()[0].write('/tmp/h115.hgr')" || exit 1
O=gpurun_out/cold_graph_ab.txt
: > $O
for r in 1 2 3; do
  for g in 1 0; do
    echo -n "graph=$g " >> $O
    timeout -k 10 200 python3 tools/cold_probe.py /tmp/h115.hgr 5 EK_LANCZOS_GRAPH=$g >> $O || exit 1
  done
done
cat $O
