cd $GRAFT_REPO_ROOT
bash tools/gpu_tests.sh r06gb2 tests/test_gpu_parity.py tests/test_gpu_scale.py -k "fallback_paths or bitmaps_off_chip or kl_bitexact" || exit $?
bash tools/step_ab.sh
