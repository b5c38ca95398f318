#!/bin/bash
# Full GPU pass: parity tests, smoke, bench (N=1), bench under torchrun (RCCL
# path at world 1), H2D pipeline rate, rocprofv3 kernel-trace summary.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-round}
step() { local name=$1; shift; "$@"; local rc=$?; echo "[$name] rc=$rc" >&2; case $rc in 0) ;; *) exit $rc;; esac; }
step tests timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1
tail -2 gpurun_out/${TAG}_tests.log
step smoke timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
cat gpurun_out/${TAG}_bench.json
step torchrun timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 5 --warmup 1 --no-cpu --no-extra > gpurun_out/${TAG}_torchrun.json 2> gpurun_out/${TAG}_torchrun.err
cat gpurun_out/${TAG}_torchrun.json
step h2d timeout -k 10 600 python tools/h2d_bench.py > gpurun_out/${TAG}_h2d.json 2> gpurun_out/${TAG}_h2d.err
cat gpurun_out/${TAG}_h2d.json
step prof timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu > gpurun_out/${TAG}_prof.log 2>&1
grep -h crc32c_tiles gpurun_out/${TAG}_prof/run_kernel_stats.csv | cut -c1-220
step pmc timeout -k 10 900 python tools/pmc_traffic.py ${ROUND:-r01} > gpurun_out/${TAG}_pmc.json 2> gpurun_out/${TAG}_pmc.err
cat gpurun_out/${TAG}_pmc.json
step mixed timeout -k 10 600 python bench.py --no-cpu --mixed --steps 5 > gpurun_out/${TAG}_mixed.json 2> gpurun_out/${TAG}_mixed.err
cat gpurun_out/${TAG}_mixed.json
