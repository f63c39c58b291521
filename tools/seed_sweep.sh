cd $GRAFT_REPO_ROOT
bash tools/gpu_tests.sh r06sw tests/test_gpu_scale.py -k "seed_sweep"
