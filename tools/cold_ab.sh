# GPU box: fresh-process wall of gKL2 -EIG on the headline: the current build,
# the current build with EK_LANCZOS_GRAPH=0, and build_old (tools/ab_build.sh
# old REV + its gKL2), alternating.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 python3 -c "
import importlib.util
spec=importlib.util.spec_from_file_location('ek','eig-kl-algorithm_amd/__init__.py'); ek=importlib.util.module_from_spec(spec); spec.loader.exec_module(ek)
ek.Hypergraph.generate(1.15,1).largest_component()[0].write('/tmp/h115.hgr')" || exit 1
O=gpurun_out/cold_ab.txt
: > $O
for r in 1 2 3; do
  echo -n "build " >> $O
  EK_COLD_BUILD=build timeout -k 10 200 python3 tools/cold_probe.py /tmp/h115.hgr 5 >> $O || exit 1
  echo -n "build_graph0 " >> $O
  EK_COLD_BUILD=build timeout -k 10 200 python3 tools/cold_probe.py /tmp/h115.hgr 5 EK_LANCZOS_GRAPH=0 >> $O || exit 1
  echo -n "build_old " >> $O
  EK_COLD_BUILD=build_old timeout -k 10 200 python3 tools/cold_probe.py /tmp/h115.hgr 5 >> $O || exit 1
done
cat $O
