set -o pipefail
# Verify: expected-CRC loads nontemporal (21), bitmap stores nontemporal (22), both (23), one process.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python tools/exp_knobs.py '[{}, {"store_policy": 21}, {"store_policy": 22}, {"store_policy": 23}]' 5 > gpurun_out/s3g.json 2> gpurun_out/s3g.err; rc=$?; cat gpurun_out/s3g.json; exit $rc
