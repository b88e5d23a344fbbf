#!/bin/bash
# round 6: LDS rows issue their payload loads before the sender sort -- drain parity (not full
# size), then interleaved runs against the previous drain source (GSP_LIB_VARIANT=old), ticks 6-25
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r06el}; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests/test_pview_drain_gpu.py -k "not full_size" -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc -ne 0 ] && exit $rc
bash scripts/ab_drain.sh ${TAG:-r06el}/ab base old | tee $OUT/ab.txt
