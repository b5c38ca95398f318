#!/bin/bash
# Round-2 GPU pass (one gpurun call): box CPU facts, parity tests, smoke,
# bench (N=1), bench under torchrun (RCCL path, world 1), optional knob A/B.
#   tools/gpu_r2.sh TAG [AB_VARIANTS_JSON]
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r2}
step() { local name=$1; shift; "$@"; local rc=$?; echo "[$name] rc=$rc" >&2; case $rc in 0) ;; *) exit $rc;; esac; }
{ echo "nproc $(nproc)"; python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)))";
  echo "cpu.max $(cat /sys/fs/cgroup/cpu.max 2>/dev/null)"; lscpu | grep -E "Model name|Socket|Thread|Core|NUMA node\(s\)"; } > gpurun_out/${TAG}_box.txt 2>&1
cat gpurun_out/${TAG}_box.txt
step tests timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
tail -2 gpurun_out/${TAG}_tests.log
step smoke timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
cat gpurun_out/${TAG}_bench.json
step torchrun timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 5 --warmup 1 --no-cpu > gpurun_out/${TAG}_torchrun.json 2> gpurun_out/${TAG}_torchrun.err
cat gpurun_out/${TAG}_torchrun.json
if [ -n "$2" ]; then
  step ab timeout -k 10 600 python tools/exp_knobs.py "$2" 4 > gpurun_out/${TAG}_ab.json 2> gpurun_out/${TAG}_ab.err
  cat gpurun_out/${TAG}_ab.json
fi
