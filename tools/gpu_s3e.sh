set -o pipefail
# SQ counters of the gather kernel with the slot protocol (policy 2) and without it (20).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python3 tools/exp_pmc_gather.py > gpurun_out/s3e_pmc.json 2> gpurun_out/s3e_pmc.err; rc=$?; cat gpurun_out/s3e_pmc.json; exit $rc
