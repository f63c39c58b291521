# GPU box: the KL stream created on first use (default) against at ek_init (EK_KSTREAM_EAGER=1): the KL/solve GPU tests, then 2 x 2 alternating cold_probe runs of 7 fresh gKL2 -EIG processes on the headline file.
# (Run once; the lazy form lost: the switch and the lazy stream were removed again, see profiles/r06/cold_kstream_ab.txt.)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/gpu_tests.sh r06ks tests/test_gpu_parity.py tests/test_gpu_scale.py -k "kl or solve_file or headline or fresh" || exit $?
timeout -k 10 120 python3 -c "
import sys; sys.path.insert(0,'tests')
from conftest import load_package
ek=load_package(); ek.Hypergraph.generate(1.15,1).largest_component()[0].write('/tmp/h115.hgr')" || exit 1
O=gpurun_out/cold_kstream_ab.txt
: > $O
for i in 1 2; do
  echo "lazy $(timeout -k 10 200 python3 tools/cold_probe.py /tmp/h115.hgr 7)" >> $O || exit 1
  echo "eager $(timeout -k 10 200 python3 tools/cold_probe.py /tmp/h115.hgr 7 EK_KSTREAM_EAGER=1)" >> $O || exit 1
done
cat $O
