# GPU box: KL build switches re-measured with 2048-position chunks: one-trip
# early rescans (EK_E_TWO_TRIPS=0) and the next pair published by P
# (EK_KL_NEXT=1), parity subset each, then the warm step A/B.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/kl_switch_ab.txt
for v in e2t0 next1; do
  EK_LIB_PATH=eig-kl-algorithm_amd/build_$v/libeigkl_hip.so timeout -k 10 600 python3 -u -m pytest -m gpu -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_scale.py -k "(kl_bitexact or fallback_paths or headline_solve or bitmaps_off_chip) and not PIPE" > gpurun_out/kl_$v.log 2>&1 || { tail -20 gpurun_out/kl_$v.log; exit 1; }
  tail -1 gpurun_out/kl_$v.log
  timeout -k 10 600 python3 tools/step_ab.py eig-kl-algorithm_amd/build/libeigkl_hip.so eig-kl-algorithm_amd/build_$v/libeigkl_hip.so 2 2>&1 | grep -v amdgpu.ids >> gpurun_out/kl_switch_ab.txt || exit 1
done
cat gpurun_out/kl_switch_ab.txt
