# GPU box: bench.py --gpus 2 on the one GPU (host-staged seam: RCCL refuses two
# ranks on one device): the N>1 code path end to end.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python3 -u bench.py --gpus 2 --steps 3 --warmup 1 > gpurun_out/n2_bench.json 2> gpurun_out/n2_bench.err
rc=$?
tail -c 1500 gpurun_out/n2_bench.json
tail -5 gpurun_out/n2_bench.err
exit $rc
