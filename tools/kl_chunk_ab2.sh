# GPU box: KL chunk 2048 / 4096 against 1024: parity subset for 4096, then the warm step, alternating.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
EK_LIB_PATH=eig-kl-algorithm_amd/build_c4096/libeigkl_hip.so timeout -k 10 600 python3 -u -m pytest -m gpu -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_scale.py -k "kl_bitexact or fallback_paths or headline_solve or bitmaps_off_chip" > gpurun_out/kl_chunk_4096.log 2>&1 || { tail -20 gpurun_out/kl_chunk_4096.log; exit 1; }
tail -1 gpurun_out/kl_chunk_4096.log
timeout -k 10 900 python3 tools/step_ab.py eig-kl-algorithm_amd/build/libeigkl_hip.so eig-kl-algorithm_amd/build_c2048/libeigkl_hip.so 4 2>&1 | grep -v amdgpu.ids > gpurun_out/kl_chunk_ab2.txt || exit 1
timeout -k 10 600 python3 tools/step_ab.py eig-kl-algorithm_amd/build/libeigkl_hip.so eig-kl-algorithm_amd/build_c4096/libeigkl_hip.so 2 2>&1 | grep -v amdgpu.ids >> gpurun_out/kl_chunk_ab2.txt || exit 1
cat gpurun_out/kl_chunk_ab2.txt
