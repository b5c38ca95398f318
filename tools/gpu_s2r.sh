set -o pipefail
# Gather slot count sensitivity (binary A/B in one process): 15 (product) vs 7 vs 3 slots.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python tools/exp_ab_libs.py build/ab/base/libhadoofus_crc32c.so build/ab/slots7/libhadoofus_crc32c.so 4 > gpurun_out/s2r_ab7.json 2> gpurun_out/s2r_ab7.err; rc=$?; cat gpurun_out/s2r_ab7.json; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python tools/exp_ab_libs.py build/ab/base/libhadoofus_crc32c.so build/ab/slots3/libhadoofus_crc32c.so 4 > gpurun_out/s2r_ab3.json 2> gpurun_out/s2r_ab3.err; rc=$?; cat gpurun_out/s2r_ab3.json; exit $rc
