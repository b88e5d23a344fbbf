#!/bin/bash
# round 6: the TFAIL send kernel (wave-built gossipable bitmaps) -- parity of every partial-view
# test file that runs TFAIL, then the variant cost again
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r06tf}; mkdir -p $OUT
timeout -k 10 800 python -u -m pytest tests/test_pview_gpu.py tests/test_pview_drain_gpu.py tests/test_policy_gpu.py tests/test_events_gpu.py -m gpu -k "not full_size" -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -ne 0 ] && exit $rc
TAG=${TAG:-r06tf} bash scripts/gpu_r06_swimcost.sh
