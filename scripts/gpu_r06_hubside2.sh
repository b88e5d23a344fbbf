#!/bin/bash
# round 6: the hub kernel on its own stream as the default -- drain / partial-view / event parity,
# then drain stats and the A/B against one stream (GSP_TEST_PV_DRAIN_STREAM=0), ticks 6-25, 6-55
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r06hs2}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_pview_drain_gpu.py tests/test_pview_gpu.py tests/test_events_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc -ne 0 ] && exit $rc
for steps in 20 50; do for v in 2 0; do
  GSP_TEST_PV_DRAIN_STREAM=$v timeout -k 10 240 python3 -u scripts/bench_pview.py --inbox 0 --steps $steps --warmup 5 --no-cpu-baseline > $OUT/ab_${steps}_$v.json 2>> $OUT/ab.err || exit 1
  python3 -c "
import json; d=json.loads(open('$OUT/ab_${steps}_$v.json').read().strip().splitlines()[-1]); dc=d['drain_classes']
print('steps $steps stream=$v tick-kernels %.3f ms  classes [%s]' % (d['roofline']['kernel_ms_per_tick'], ' '.join('%.3f' % c['kernel_ms_per_tick'] for c in dc)))" | tee -a $OUT/ab.txt
done; done
