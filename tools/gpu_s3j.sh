set -o pipefail
# Gather slot protocol committed after the slot's refill loads (late) vs in finish (product), binary A/B both ways.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python tools/exp_ab_libs.py build/ab/base/libhadoofus_crc32c.so build/ab/late/libhadoofus_crc32c.so 4 > gpurun_out/s3j_ab.json 2> gpurun_out/s3j_ab.err; rc=$?; cat gpurun_out/s3j_ab.json; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python tools/exp_ab_libs.py build/ab/late/libhadoofus_crc32c.so build/ab/base/libhadoofus_crc32c.so 4 > gpurun_out/s3j_ba.json 2> gpurun_out/s3j_ba.err; rc=$?; cat gpurun_out/s3j_ba.json; exit $rc
