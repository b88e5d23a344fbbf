#!/bin/bash
# round 6: the full-size drain-all tests (config 5 at 1,048,576 nodes) and the rowx posted-size
# policy test, each under its own limit
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r06full}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_pview_drain_gpu.py -k full_size -x -v -s --timeout 600 --timeout-method thread > $OUT/full.log 2>&1
rc=$?; tail -6 $OUT/full.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -m pytest tests/test_policy_gpu.py -k posted -x -v --timeout 240 --timeout-method thread > $OUT/posted.log 2>&1
rc=$?; tail -4 $OUT/posted.log; exit $rc
