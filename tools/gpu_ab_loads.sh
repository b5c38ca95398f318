#!/bin/bash
# Shape parity (all shapes incl. buffer loads), then in-process A/B of the
# global-load vs buffer-load forms of the default shape.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-loads}
timeout -k 10 600 python -u -m pytest tests/test_gpu_shapes.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_tests.log; echo "tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
AB_VARIANTS=${AB_VARIANTS:-"3,1,3,3;3,2,3,3"} timeout -k 10 900 python -u tools/exp_ab.py > gpurun_out/${TAG}_ab.json 2> gpurun_out/${TAG}_ab.err
rc=$?; echo "ab rc=$rc"; cut -c1-1500 gpurun_out/${TAG}_ab.json; exit $rc
