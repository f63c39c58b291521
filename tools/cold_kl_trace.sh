# GPU box: one fresh gKL2 -EIG run on the headline with the host phase trace
# (EK_TRACE) and the cold stamps, with and without the Lanczos graphs.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out /tmp/ekck
timeout -k 10 120 python3 -c "
import importlib.util
spec=importlib.util.spec_from_file_location('ek','eig-kl-algorithm_amd/__init__.py'); ek=importlib.util.module_from_spec(spec); spec.loader.exec_module(ek)
ek.Hypergraph.generate(1.15,1).largest_component()[0].write('/tmp/h115.hgr')" || exit 1
: > $GRAFT_REPO_ROOT/gpurun_out/cold_kl_trace.txt
cd /tmp/ekck
for g in 1 0; do
  echo "=== EK_LANCZOS_GRAPH=$g" >> $GRAFT_REPO_ROOT/gpurun_out/cold_kl_trace.txt
  EK_LANCZOS_GRAPH=$g EK_TRACE=1 EK_COLD_TRACE=1 timeout -k 10 60 $GRAFT_REPO_ROOT/eig-kl-algorithm_amd/build/bin/gKL2 /tmp/h115.hgr -EIG --quiet >> $GRAFT_REPO_ROOT/gpurun_out/cold_kl_trace.txt 2>&1 || exit 1
done
cat $GRAFT_REPO_ROOT/gpurun_out/cold_kl_trace.txt | grep -v "^\[lanczos\]" | head -120
