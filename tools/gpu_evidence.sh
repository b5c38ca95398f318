#!/bin/bash
# Round evidence pass (one gpurun call): parity tests, smoke, the driver's
# bench line, bench under rocprofv3 (kernel trace + stats), HBM traffic from
# PMC passes, the RCCL path at world 1, the C4 config, device-stream and
# small-call latency benches.   tools/gpu_evidence.sh TAG ROUND
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-ev}
RND=${2:-r03}
O=gpurun_out/${TAG}
step() { local name=$1; shift; "$@"; local rc=$?; echo "[$name] rc=$rc" >&2; case $rc in 0) ;; *) exit $rc;; esac; }
step tests timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > ${O}_tests.log 2>&1
tail -2 ${O}_tests.log
step smoke timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench timeout -k 10 600 python bench.py > ${O}_bench.json 2> ${O}_bench.err
cat ${O}_bench.json
step prof timeout -k 10 600 rocprofv3 --kernel-trace --stats -d ${O}_prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu > ${O}_prof.log 2>&1
grep -h crc32c_tiles ${O}_prof/run_kernel_stats.csv | cut -c1-200
step pmc timeout -k 10 900 python tools/pmc_traffic.py ${RND} > ${O}_pmc.json 2> ${O}_pmc.err
cat ${O}_pmc.json
step torchrun timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 5 --warmup 1 --no-cpu > ${O}_torchrun.json 2> ${O}_torchrun.err
cat ${O}_torchrun.json
step c4 timeout -k 10 600 python bench.py --config C4 --steps 10 --no-cpu > ${O}_c4.json 2> ${O}_c4.err
cat ${O}_c4.json
step dstream timeout -k 10 300 python tools/device_stream_bench.py > ${O}_dstream.json 2> ${O}_dstream.err
cat ${O}_dstream.json
step small timeout -k 10 300 python tools/small_launch.py > ${O}_small.json 2> ${O}_small.err
cat ${O}_small.json
