# GPU box: the Lanczos solve at the headline with the step's vector outputs
# stored plainly, non-temporally and write-through (EK_OUT_STORE builds).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
EK_AB_ROUNDS=3 timeout -k 10 600 python3 tools/lib_ab.py eig-kl-algorithm_amd/build/libeigkl_hip.so eig-kl-algorithm_amd/build_nt/libeigkl_hip.so lcc1.15 > gpurun_out/out_store_ab.txt 2>&1 || exit 1
EK_AB_ROUNDS=2 timeout -k 10 600 python3 tools/lib_ab.py eig-kl-algorithm_amd/build/libeigkl_hip.so eig-kl-algorithm_amd/build_sc1/libeigkl_hip.so lcc1.15 >> gpurun_out/out_store_ab.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/out_store_ab.txt
