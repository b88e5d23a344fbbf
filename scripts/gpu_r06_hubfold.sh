#!/bin/bash
# round 6: the hub kernel's fold staged in LDS -- drain parity (hub and full-size cases
# included), then interleaved runs against the previous drain source over ticks 6-75 and 6-25
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r06hf}; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests/test_pview_drain_gpu.py -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc -ne 0 ] && exit $rc
for steps in 70 20; do for v in new old new old; do
  VAR=""; [ $v = old ] && VAR=old
  GSP_LIB_VARIANT=$VAR timeout -k 10 240 python3 -u scripts/bench_pview.py --inbox 0 --steps $steps --warmup 5 --no-cpu-baseline > $OUT/ab.json 2>> $OUT/ab.err || exit 1
  python3 -c "
import json; d=json.loads(open('$OUT/ab.json').read().strip().splitlines()[-1]); dc=d['drain_classes']
print('steps $steps $v tick-kernels %.3f ms  hub %.3f ms' % (d['roofline']['kernel_ms_per_tick'], dc[-1]['kernel_ms_per_tick']))" | tee -a $OUT/ab.txt
done; done
