#!/bin/bash
# Shape experiment: parity of every tiled-kernel shape, then in-process A/B
# timing of the candidate shapes (tools/exp_ab.py).  Stops on any failure.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-shapes}
timeout -k 10 600 python -u -m pytest tests/test_gpu_shapes.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_tests.log; echo "tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
AB_VARIANTS=${AB_VARIANTS:-"3,1,3,3;3,1,2,3,2,1024;3,1,3,3,2,1024;3,1,3,3,2,768;3,1,3,3,2,512;3,1,2,3,4,512;3,1,3,3,1,768"} \
  timeout -k 10 900 python -u tools/exp_ab.py > gpurun_out/${TAG}_ab.json 2> gpurun_out/${TAG}_ab.err
rc=$?; echo "ab rc=$rc"; cat gpurun_out/${TAG}_ab.json | cut -c1-3000; exit $rc
