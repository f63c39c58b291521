cd $GRAFT_REPO_ROOT
O=gpurun_out/r06w_chkfold_ab.txt
timeout -k 10 300 python3 tools/env_ab.py EK_CHK_FOLD 1 0 3 2>&1 | grep -v amdgpu.ids > $O || exit 1
cat $O
bash tools/gpu_tests.sh r06w tests/test_gpu_parity.py tests/test_gpu_scale.py -k "lanczos or headline or solve"
