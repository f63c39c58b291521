# GPU box: the warm step through the default build and the max-ilp scheduler build (KL us/swap).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python3 tools/step_ab.py eig-kl-algorithm_amd/build/libeigkl_hip.so eig-kl-algorithm_amd/build_ilp/libeigkl_hip.so 3 2>&1 | grep -v amdgpu.ids > gpurun_out/sched_ab.txt
rc=$?
cat gpurun_out/sched_ab.txt
exit $rc
