set -o pipefail
# Gather slot ordering by compiler barriers only vs LDS fences (binary A/B both ways), and the
# group-store cache policies re-measured on the pipelined gather kernel.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python tools/exp_ab_libs.py build/ab/base/libhadoofus_crc32c.so build/ab/asmbar/libhadoofus_crc32c.so 4 > gpurun_out/s2v_ab.json 2> gpurun_out/s2v_ab.err; rc=$?; cat gpurun_out/s2v_ab.json; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python tools/exp_ab_libs.py build/ab/asmbar/libhadoofus_crc32c.so build/ab/base/libhadoofus_crc32c.so 4 > gpurun_out/s2v_ba.json 2> gpurun_out/s2v_ba.err; rc=$?; cat gpurun_out/s2v_ba.json; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python tools/exp_knobs.py '[{}, {"store_policy": 1}, {"store_policy": 7}, {"store_policy": 6}]' 4 > gpurun_out/s2v_knobs.json 2> gpurun_out/s2v_knobs.err; rc=$?; cat gpurun_out/s2v_knobs.json; exit $rc
