# GPU box: the 10x -EIG file path and the headline step with 12 / 14 / 16 KL
# adjacency threads (EK_KL_GRAPH_THREADS).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
O=gpurun_out/pipe10_threads.txt
: > $O
for t in 12 16 14; do
  echo "EK_KL_GRAPH_THREADS=$t" >> $O
  EK_KL_GRAPH_THREADS=$t timeout -k 10 300 python3 tools/pipe10.py 2>&1 | grep "^wall" >> $O || exit 1
done
timeout -k 10 600 python3 tools/step_ab.py EK_KL_GRAPH_THREADS=12 EK_KL_GRAPH_THREADS=16 2 2>&1 | grep -v amdgpu.ids >> $O || exit 1
cat $O
