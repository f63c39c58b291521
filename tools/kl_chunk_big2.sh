# GPU box: the KL rate by graph size, 2048 (default) against 4096 chunks.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
O=gpurun_out/kl_chunk_big2.txt
echo "chunk 2048" > $O
timeout -k 10 500 python3 tools/kl_big.py 2>&1 | grep -v amdgpu.ids >> $O || exit 1
echo "chunk 4096" >> $O
EK_LIB_PATH=eig-kl-algorithm_amd/build_c4096/libeigkl_hip.so timeout -k 10 500 python3 tools/kl_big.py 2>&1 | grep -v amdgpu.ids >> $O || exit 1
cat $O
