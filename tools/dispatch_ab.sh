cd $GRAFT_REPO_ROOT
O=gpurun_out/r06r_ab.txt
timeout -k 10 300 python3 tools/env_ab.py EK_PRO_TICKETS "" 0 2 2>&1 | grep -v amdgpu.ids > $O || exit 1
EK_AB_10X=1 timeout -k 10 400 python3 tools/env_ab.py EK_PRO_TICKETS "" 0 1 2>&1 | grep -v amdgpu.ids >> $O || exit 1
cat $O
bash tools/gpu_tests.sh r06r tests/test_gpu_parity.py -k "dispatch_order or lanczos_golden or partial_reorth or device_paths"
