#!/bin/bash
# Laplacian-build A/B (through gpurun from the repo root): rocprofv3
# --kernel-trace over tools/build_lab.py (the device build alone, 1x and 10x
# synthetic) with each library build given.  usage: tools/rows_ab.sh build_dir...
# Output: gpurun_out/rp_ab_<build_dir>/.
set -e
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd /tmp && export TMPDIR=/tmp
for b in "$@"; do
  export EK_LIB_PATH=$R/eig-kl-algorithm_amd/$b/libeigkl_hip.so
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/rp_ab_$b" -o p -- \
      python3 "$R/tools/build_lab.py" > "$R/gpurun_out/rp_ab_$b.txt" 2>&1
done
echo done
