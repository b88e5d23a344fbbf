#!/bin/bash
# round 6: drain classes on a second stream beside the split kernels -- drain parity, then two
# interleaved runs with the side stream on and off (GSP_TEST_PV_DRAIN_STREAM=0), ticks 6-25
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r06ds}; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests/test_pview_drain_gpu.py tests/test_pview_gpu.py -k "drain or nowait or inbox" -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do for v in 1 0; do
  GSP_TEST_PV_DRAIN_STREAM=$v timeout -k 10 200 python3 -u scripts/bench_pview.py --inbox 0 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/ab_${v}_$rep.json 2>> $OUT/ab.err || exit 1
  python3 -c "
import json; d=json.loads(open('$OUT/ab_${v}_$rep.json').read().strip().splitlines()[-1]); dc=d['drain_classes']
print('stream=$v rep$rep step %.3f ms tick-kernels %.3f ms drain-classes %.3f ms' % (d['ms_per_step'], d['roofline']['kernel_ms_per_tick'], sum(c['kernel_ms_per_tick'] for c in dc)))" | tee -a $OUT/ab.txt
done; done
