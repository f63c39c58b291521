# GPU box: the device Laplacian build after the register sort of short rows:
# (Run once: the register form measured slower and was reverted; profiles/r06/rows_regsort_ab.txt.)
# its bit-identity tests (device vs host build), the headline file path, then
# kernel traces of the bench's headline probe (1 untimed + 3 solve_file
# steps) with this build and, when present, an A/B build (EK_LIB_PATH).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/gpu_tests.sh r06rows tests/test_gpu_build.py tests/test_gpu_scale.py -k "build or headline or solve_file or seed_sweep" || exit $?
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/rows_prof -o rows -- python3 $R/tools/spmv_probe.py file 1.15lcc 1 1 3 > $R/gpurun_out/rows_prof.log 2>&1 || exit $?
if [ -f $R/eig-kl-algorithm_amd/build_rowsold/libeigkl_hip.so ]; then
  EK_LIB_PATH=$R/eig-kl-algorithm_amd/build_rowsold/libeigkl_hip.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/rows_prof_old -o rows -- python3 $R/tools/spmv_probe.py file 1.15lcc 1 1 3 > $R/gpurun_out/rows_prof_old.log 2>&1 || exit $?
fi
cd $R
for d in rows_prof rows_prof_old; do
  f=$(find gpurun_out/$d -name "*kernel_stats.csv" 2>/dev/null | head -1)
  [ -n "$f" ] && { echo "== $d"; grep -E "k_rows|k_row_write" "$f"; }
done
exit 0
