# GPU box: the KL loop's fixed LDS layout: KL parity subset, then the warm step A/B (EK_KL_FIXLDS 1 vs 0).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/gpu_tests.sh r06fix tests/test_gpu_parity.py tests/test_gpu_scale.py -k "kl_bitexact or fallback_paths or bitmaps_off_chip or headline_solve or seed_sweep" || exit $?
timeout -k 10 600 python3 tools/step_ab.py EK_KL_FIXLDS=1 EK_KL_FIXLDS=0 3 2>&1 | grep -v amdgpu.ids > gpurun_out/kl_fix_ab.txt || exit 1
cat gpurun_out/kl_fix_ab.txt
