#!/bin/bash
# Round evidence pass (one gpurun call): parity tests, smoke, the driver's
# bench line, bench under rocprofv3 (kernel trace + stats), HBM traffic from
# PMC passes, the RCCL path at world 1, the C4 config, device-stream and
# small-call latency benches.   tools/gpu_evidence.sh TAG ROUND [PARTS]
# PARTS: any of t (tests + smoke), b (bench, and the same command under
# rocprofv3 with its trace-vs-line comparison), p (PMC + torchrun +
# C4), d (device-stream + small-call benches), q (SQ/TA/TCP counters of the
# compute and verify kernels, tools/pmc_sq.py), s (phase stamps of the
# speculative verify, tools/spec_phases.py), r (reader / copy costs:
# tools/reader_sizes.py, reader_calls.py, copy_phases.py), j (job
# coalescing on/off, tools/jobs_coalesce_ab.py), m (streams sharing the
# mailbox's hardware queue, tools/mb_queue_share.py); default tbpd, one call.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-ev}
RND=${2:-r03}
PARTS=${3:-tbpd}
O=gpurun_out/${TAG}
has() { case $PARTS in *$1*) return 0;; esac; return 1; }
step() { local name=$1; shift; "$@"; local rc=$?; echo "[$name] rc=$rc" >&2; case $rc in 0) ;; *) exit $rc;; esac; }
has t && step tests timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > ${O}_tests.log 2>&1
has t && tail -2 ${O}_tests.log
has t && step smoke timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()"
has b && step bench timeout -k 10 600 python bench.py > ${O}_bench.json 2> ${O}_bench.err
has b && cat ${O}_bench.json
# the driver's own command under the profiler: its bench line and its trace
# come from one process (tools/trace_vs_line.py compares the timed launches)
has b && step prof timeout -k 10 900 rocprofv3 --kernel-trace --stats -d ${O}_prof -o run --output-format csv -- python3 bench.py > ${O}_prof.log 2>&1
has b && step trace_vs_line python tools/trace_vs_line.py ${O}_prof/run_kernel_trace.csv ${O}_prof.log ${O}_trace_vs_line.json
has b && grep -h crc32c_tiles ${O}_prof/run_kernel_stats.csv | cut -c1-200
has p && step pmc timeout -k 10 900 python tools/pmc_traffic.py ${RND} > ${O}_pmc.json 2> ${O}_pmc.err
has p && cat ${O}_pmc.json
has p && step torchrun timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 5 --warmup 1 --no-cpu > ${O}_torchrun.json 2> ${O}_torchrun.err
has p && cat ${O}_torchrun.json
has p && step c4 timeout -k 10 600 python bench.py --config C4 --steps 10 --no-cpu > ${O}_c4.json 2> ${O}_c4.err
has p && cat ${O}_c4.json
has d && step dstream timeout -k 10 300 python tools/device_stream_bench.py > ${O}_dstream.json 2> ${O}_dstream.err
has d && cat ${O}_dstream.json
has d && step small timeout -k 10 300 python tools/small_launch.py > ${O}_small.json 2> ${O}_small.err
has d && cat ${O}_small.json
has q && step pmc_sq timeout -k 10 900 python tools/pmc_sq.py ${O}_pmc_sq.json > /dev/null 2> ${O}_pmc_sq.err
has q && cat ${O}_pmc_sq.json
has s && step spec_phases timeout -k 10 300 python tools/spec_phases.py ${O}_spec_phases.json > /dev/null 2> ${O}_spec_phases.err
has s && cat ${O}_spec_phases.json
has r && step reader_sizes timeout -k 10 300 python tools/reader_sizes.py ${O}_reader_sizes.json > /dev/null 2> ${O}_reader_sizes.err
has r && step reader_calls timeout -k 10 300 python tools/reader_calls.py ${O}_reader_calls.json > /dev/null 2> ${O}_reader_calls.err
has r && step copy_phases timeout -k 10 300 python tools/copy_phases.py ${O}_copy_phases.json > /dev/null 2> ${O}_copy_phases.err
has j && step jobs_ab timeout -k 10 300 python tools/jobs_coalesce_ab.py ${O}_jobs_ab.json > /dev/null 2> ${O}_jobs_ab.err
has j && cat ${O}_jobs_ab.json | tail -3
has m && step mb_share timeout -k 10 300 python tools/mb_queue_share.py ${O}_mb_share.json > ${O}_mb_share.log 2>&1
has m && cat ${O}_mb_share.log
exit 0
