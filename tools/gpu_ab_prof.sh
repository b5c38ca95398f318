#!/bin/bash
# Kernel traces of tools/device_stream_bench.py for several builds on one box:
#   tools/gpu_ab_prof.sh NAME ...   (build/ab/NAME/libhadoofus_crc32c.so; "tree" = this tree's library)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
for n in "$@"; do
  lib=build/ab/$n/libhadoofus_crc32c.so; [ "$n" = tree ] && lib=
  DSB_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/abp_$n -o run --output-format csv \
    -- python3 tools/device_stream_bench.py > gpurun_out/abp_$n.log 2>&1 || exit $?
done
