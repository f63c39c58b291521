cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python3 -u tools/parity_sweep.py > gpurun_out/parity_sweep.txt 2>&1
rc=$?
grep -v amdgpu.ids gpurun_out/parity_sweep.txt | tail -40
exit $rc
