#!/bin/bash
# round 6: the hub kernel alone on a side stream (GSP_TEST_PV_DRAIN_STREAM=2) against one
# stream -- drain parity in that mode, then interleaved runs over ticks 6-25 and 6-55
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r06hs}; mkdir -p $OUT
GSP_TEST_PV_DRAIN_STREAM=2 timeout -k 10 600 python -u -m pytest tests/test_pview_drain_gpu.py -k "not full_size" -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc -ne 0 ] && exit $rc
for steps in 20 50; do for rep in 1 2; do for v in 0 2; do
  GSP_TEST_PV_DRAIN_STREAM=$v timeout -k 10 240 python3 -u scripts/bench_pview.py --inbox 0 --steps $steps --warmup 5 --no-cpu-baseline > $OUT/ab_${steps}_${v}_$rep.json 2>> $OUT/ab.err || exit 1
  python3 -c "
import json; d=json.loads(open('$OUT/ab_${steps}_${v}_$rep.json').read().strip().splitlines()[-1])
print('steps $steps side=$v rep$rep step %.3f ms tick-kernels %.3f ms' % (d['ms_per_step'], d['roofline']['kernel_ms_per_tick']))" | tee -a $OUT/ab.txt
done; done; done
