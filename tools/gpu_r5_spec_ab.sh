#!/bin/bash
# Round 5: the speculative kernel's prologue / pool changes on one box.
# Tests of the packet paths, then phase stamps (tools/spec_phases.py) of the
# base and new diagnostic builds and of the new one at pool thresholds 32 and
# 4, then device-stream rates of the base and new product builds interleaved.
#   tools/gpu_r5_spec_ab.sh TAG BASE_DIR
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r5g}
BASE=${2:-build/ab/r5base}
timeout -k 10 600 python -u -m pytest tests/test_spec_verify.py tests/test_packets.py tests/test_read_host.py -m gpu -q -x \
  -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
tail -2 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
summ() {
  python -c "
import json,statistics as st,sys
d=json.load(open(sys.argv[1]))
for k,v in d.items():
    rs=v['runs']
    print(sys.argv[2], k, 'p1', st.median(r['p1_us'][1] for r in rs), 'p4', st.median(r['p4_us'][0] for r in rs),
          'p3max', st.median(r['p3_us'][2] for r in rs), 'loop_end_max', st.median(r['wave_loop_end_us'][2] for r in rs))
" "$1" "$2"
}
for rep in 1 2; do
  SPH_LIB=$BASE/libhadoofus_crc32c_diag.so timeout -k 10 120 python tools/spec_phases.py gpurun_out/${TAG}_ph_base_$rep.json > /dev/null 2>> gpurun_out/${TAG}.err || exit $?
  summ gpurun_out/${TAG}_ph_base_$rep.json base
  timeout -k 10 120 python tools/spec_phases.py gpurun_out/${TAG}_ph_new_$rep.json > /dev/null 2>> gpurun_out/${TAG}.err || exit $?
  summ gpurun_out/${TAG}_ph_new_$rep.json new
  HDFS_CRC32C_SPEC_POOL=4 timeout -k 10 120 python tools/spec_phases.py gpurun_out/${TAG}_ph_new4_$rep.json > /dev/null 2>> gpurun_out/${TAG}.err || exit $?
  summ gpurun_out/${TAG}_ph_new4_$rep.json new_pool4
done
for i in 1 2; do
  DSB_LIB=$BASE/libhadoofus_crc32c.so timeout -k 10 300 python tools/device_stream_bench.py > gpurun_out/${TAG}_ds_base$i.json 2>> gpurun_out/${TAG}.err || exit $?
  timeout -k 10 300 python tools/device_stream_bench.py > gpurun_out/${TAG}_ds_new$i.json 2>> gpurun_out/${TAG}.err || exit $?
  python -c "
import json
for n in ('base','new'):
    d=json.load(open('gpurun_out/${TAG}_ds_'+n+'$i.json'))
    print(n, 'run_1GiB', d['run_1GiB']['us'], 'block', d['block_128MiB']['us'])
"
done
