cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
EK_TRACE=1 timeout -k 10 300 python3 tools/pipe10.py > gpurun_out/pipe10.txt 2>&1
rc=$?
grep -v amdgpu.ids gpurun_out/pipe10.txt | grep -v "^\[lanczos\]" | tail -60
exit $rc
