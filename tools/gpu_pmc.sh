#!/bin/bash
# rocprofv3 PMC passes on the verify bench (separate passes, kernel-trace only
# alongside; never combined with sys/runtime traces).  Stops on a fault/timeout.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-pmc}
ARGS="--steps 3 --warmup 1 --no-cpu --no-extra --blocks ${BLOCKS:-512}"
timeout -k 10 120 rocprofv3 -L > gpurun_out/${TAG}_counters.txt 2>&1
run() {
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" -d gpurun_out/${TAG}_$name -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/${TAG}_$name.log 2>&1
  local rc=$?
  echo "pass $name rc=$rc"
  case $rc in 124|134|137|139) exit $rc;; esac
}
run clk GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY
run fetch FETCH_SIZE
run write WRITE_SIZE
run lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS
exit 0
