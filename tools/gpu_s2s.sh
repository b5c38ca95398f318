set -o pipefail
# Late result stores (issued after the slot's refill loads) vs the product, binary A/B in one process.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python tools/exp_ab_libs.py build/ab/base/libhadoofus_crc32c.so build/ab/late/libhadoofus_crc32c.so 5 > gpurun_out/s2s_ab.json 2> gpurun_out/s2s_ab.err; rc=$?; cat gpurun_out/s2s_ab.json; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python tools/exp_ab_libs.py build/ab/late/libhadoofus_crc32c.so build/ab/base/libhadoofus_crc32c.so 5 > gpurun_out/s2s_ba.json 2> gpurun_out/s2s_ba.err; rc=$?; cat gpurun_out/s2s_ba.json; exit $rc
