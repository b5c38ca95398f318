set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python tools/exp_knobs.py '[{}, {"store_policy": 1}, {"store_policy": 6}, {"store_policy": 7}, {"store_policy": 8}, {"store_policy": 11}]' 3 > gpurun_out/s2n_knobs.json 2> gpurun_out/s2n_knobs.err; rc=$?; cat gpurun_out/s2n_knobs.json; exit $rc
