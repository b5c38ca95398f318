set -o pipefail
# Compute-mode CRC writes: XCD-split dealing (8 separate sweep windows) and a
# scattered group-store diagnostic vs the product dealing, one process.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python tools/exp_knobs.py '[{}, {"xcd_major": 2}, {"store_policy": 14}, {"xcd_major": 2, "store_policy": 14}, {"xcd_major": 0}]' 4 > gpurun_out/s2o_knobs.json 2> gpurun_out/s2o_knobs.err; rc=$?; cat gpurun_out/s2o_knobs.json; exit $rc
