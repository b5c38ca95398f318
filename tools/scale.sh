#!/usr/bin/env bash
# C4 strong scaling on one node: the 64 GiB workload (512 x 128 MiB blocks)
# split evenly over N = 1, 2, 4, 8 ranks, one process per GPU launched by
# torch.distributed.run (RCCL over xGMI for the one all-reduce of counters
# and time; no data-path collective -- independent chunks,
# src/datanode.c:2945-2954).  Prints one bench.py JSON line per N.  Needs an
# 8-GPU node (the driver's; the 1-GPU prediction is bench.py's
# extra.c4_speedup_bound).
#   tools/scale.sh [steps] [warmup]
set -euo pipefail
cd "$(dirname "$0")/.."
steps=${1:-20}
warmup=${2:-3}
ngpu=$(python3 -c "import torch; print(torch.cuda.device_count())")
for n in 1 2 4 8; do
  if [ "$n" -gt "$ngpu" ]; then
    echo "{\"skipped\": \"N=$n needs $n GPUs, $ngpu visible\"}"
    continue
  fi
  timeout -k 10 900 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node "$n" --master-addr 127.0.0.1 \
    --master-port $((29500 + n)) bench.py --gpus "$n" --steps "$steps" --warmup "$warmup" --config C4 --no-cpu \
    --no-extra | grep '^{'
done
