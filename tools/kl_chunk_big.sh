# GPU box: the KL rate by graph size, the 1024 (default) and 2048 chunk builds.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
O=gpurun_out/kl_chunk_big.txt
echo "chunk 1024" > $O
timeout -k 10 500 python3 tools/kl_big.py 2>&1 | grep -v amdgpu.ids >> $O || exit 1
echo "chunk 2048" >> $O
EK_LIB_PATH=eig-kl-algorithm_amd/build_c2048/libeigkl_hip.so timeout -k 10 500 python3 tools/kl_big.py 2>&1 | grep -v amdgpu.ids >> $O || exit 1
cat $O
