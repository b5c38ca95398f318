set -o pipefail
# Where compute mode's CRC-write cost sits, gather schedule, one process:
# product vs group stores into an L2-resident 256 KiB window (15) vs group
# stores dropped (2).  Then the bench (LDS-DMA probes in the ceiling list).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python tools/exp_knobs.py '[{}, {"store_policy": 15}, {"store_policy": 2}]' 4 > gpurun_out/s2p_knobs.json 2> gpurun_out/s2p_knobs.err; rc=$?; cat gpurun_out/s2p_knobs.json; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/s2p_bench.json 2> gpurun_out/s2p_bench.err; rc=$?; cat gpurun_out/s2p_bench.json; exit $rc
