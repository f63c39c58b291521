# GPU box: the warm step, this build against build_old (tools/ab_build.sh old REV), alternating.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python3 tools/step_ab.py eig-kl-algorithm_amd/build/libeigkl_hip.so eig-kl-algorithm_amd/build_old/libeigkl_hip.so 3 2>&1 | grep -v amdgpu.ids > gpurun_out/step_ab.txt
rc=$?
cat gpurun_out/step_ab.txt
exit $rc
