set -o pipefail
# Pair gather (two tile streams, one slot-protocol step per two tiles) vs the single-stream gather, one process;
# round buffers 2 and 3.  exp_knobs also checks the full-size CRC arrays agree across variants.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python tools/exp_knobs.py '[{}, {"runs": 3}]' 4 > gpurun_out/s3b_d2.json 2> gpurun_out/s3b_d2.err; rc=$?; cat gpurun_out/s3b_d2.json; [ $rc = 0 ] || exit $rc
HDFS_CRC32C_PAIR_DEPTH=3 timeout -k 10 600 python tools/exp_knobs.py '[{}, {"runs": 3}]' 4 > gpurun_out/s3b_d3.json 2> gpurun_out/s3b_d3.err; rc=$?; cat gpurun_out/s3b_d3.json; exit $rc
