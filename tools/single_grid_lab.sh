cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 240 python3 tools/single_grid_lab.py 2>&1 | grep -v amdgpu.ids > gpurun_out/single_grid_lab.txt
rc=$?
cat gpurun_out/single_grid_lab.txt
exit $rc
