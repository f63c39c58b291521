cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python3 tools/kl_big.py > gpurun_out/kl_big.txt 2>&1
rc=$?
cat gpurun_out/kl_big.txt | grep -v amdgpu.ids
exit $rc
