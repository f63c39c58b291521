# GPU box: the 2048-position KL chunks as the default build: KL / solve / scale subset.
cd $GRAFT_REPO_ROOT
bash tools/gpu_tests.sh r06ch tests/test_gpu_parity.py tests/test_gpu_scale.py -k "kl or split or solve or headline or seed_sweep or bitmaps"
