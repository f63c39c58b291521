# GPU box: the device split / KL / solve / CLI subset (radix-select split,
# KL adjacency started before the context is asked for).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/gpu_tests.sh r06z tests/test_gpu_scale.py tests/test_gpu_parity.py tests/test_multirank_gpu.py -k "split or kl or solve or cli or results or headline or rank"
