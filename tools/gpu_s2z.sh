set -o pipefail
# Schedule 4 with 4-tile runs (one 128-B CRC line per wave run, no cross-wave gather) vs 8-tile runs vs the gather.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python tools/exp_knobs.py '[{}, {"runs": 1}, {"runs": 1, "group_shift": 2}, {"runs": 1, "group_shift": 1}]' 4 > gpurun_out/s2z_knobs.json 2> gpurun_out/s2z_knobs.err; rc=$?; cat gpurun_out/s2z_knobs.json; exit $rc
