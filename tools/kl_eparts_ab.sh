# GPU box: E_PARTS 1 (5 gain waves) against 2: KL parity subset, the warm step A/B, the rate by size.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
EK_LIB_PATH=eig-kl-algorithm_amd/build_e1/libeigkl_hip.so timeout -k 10 600 python3 -u -m pytest -m gpu -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_scale.py -k "kl_bitexact or fallback_paths or headline_solve or bitmaps_off_chip" > gpurun_out/kl_e1.log 2>&1 || { tail -20 gpurun_out/kl_e1.log; exit 1; }
tail -1 gpurun_out/kl_e1.log
timeout -k 10 600 python3 tools/step_ab.py eig-kl-algorithm_amd/build/libeigkl_hip.so eig-kl-algorithm_amd/build_e1/libeigkl_hip.so 3 2>&1 | grep -v amdgpu.ids > gpurun_out/kl_eparts_ab.txt || exit 1
cat gpurun_out/kl_eparts_ab.txt
