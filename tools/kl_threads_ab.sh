# GPU box: the KL loop with 12 / 16 waves (EK_KL_THREADS builds) against 8: parity subset, warm step A/B.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/kl_threads_ab.txt
for t in 768 1024; do
  EK_LIB_PATH=eig-kl-algorithm_amd/build_t$t/libeigkl_hip.so timeout -k 10 600 python3 -u -m pytest -m gpu -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_scale.py -k "(kl_bitexact or fallback_paths or headline_solve or bitmaps_off_chip) and not PIPE" > gpurun_out/kl_t$t.log 2>&1 || { tail -20 gpurun_out/kl_t$t.log; exit 1; }
  tail -1 gpurun_out/kl_t$t.log
  timeout -k 10 600 python3 tools/step_ab.py eig-kl-algorithm_amd/build/libeigkl_hip.so eig-kl-algorithm_amd/build_t$t/libeigkl_hip.so 2 2>&1 | grep -v amdgpu.ids >> gpurun_out/kl_threads_ab.txt || exit 1
done
cat gpurun_out/kl_threads_ab.txt
