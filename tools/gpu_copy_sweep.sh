#!/bin/bash
# Copy-launch shapes (diagnostic build knobs): fewest units per workgroup x
# piece table in pinned or device memory, each a fresh process running
# tools/copy_phases.py.  Output: gpurun_out/$1_copy_sweep/<units>_<devtab>.json
set -e
tag=${1:-sweep}
mkdir -p gpurun_out/${tag}_copy_sweep
for u in 1024 2048 4096 8192; do
  for t in 0 1; do
    HDFS_CRC32C_COPY_WG_UNITS=$u HDFS_CRC32C_COPY_DEV_TAB=$t timeout -k 10 120 \
      python tools/copy_phases.py gpurun_out/${tag}_copy_sweep/${u}_${t}.json > /dev/null
    echo "done $u $t"
  done
done
