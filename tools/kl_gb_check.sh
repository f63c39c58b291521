# GPU box: the KL bitmaps-off-chip form: its bit-identity tests, then the rate
# by graph size (tools/kl_big.py).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/gpu_tests.sh r06gb tests/test_gpu_parity.py tests/test_gpu_scale.py -k "fallback_paths or bitmaps_off_chip or kl_bitexact" || exit $?
timeout -k 10 500 python3 tools/kl_big.py > gpurun_out/kl_big_gb.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/kl_big_gb.txt
