set -o pipefail
# Where the rest of compute mode's gap to verify sits: stores dropped on the gather vs on per-tile stores.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python tools/exp_knobs.py '[{}, {"store_policy": 2}, {"runs": 0, "store_policy": 2}, {"runs": 0}]' 4 > gpurun_out/s2x_knobs.json 2> gpurun_out/s2x_knobs.err; rc=$?; cat gpurun_out/s2x_knobs.json; exit $rc
