#!/bin/bash
# round 6: row shards without the per-tick host wait -- parity (nowait test, shard tests, the
# full-size 8-shard drain test), then an A/B of nowait against exact grids on an in-process
# group of 8 shards at config 5 (drain all and inbox 7)
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r06nw}; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests/test_pview_gpu.py tests/test_pview_drain_gpu.py -k "nowait or shards" -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -4 $OUT/tests.log; [ $rc -ne 0 ] && exit $rc
for ib in 0 7; do
  for nw in 1 0 1 0; do
    GSP_TEST_PV_NOWAIT=$nw timeout -k 10 200 python3 -u scripts/bench_pview.py --inbox $ib --group 8 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/ab_${ib}_${nw}.json 2>> $OUT/ab.err || exit 1
    python3 -c "
import json,sys; d=json.loads(open('$OUT/ab_${ib}_${nw}.json').read().strip().splitlines()[-1])
print('inbox $ib nowait $nw  step %.3f ms  kernels %.3f ms  csr %.3f ms' % (d['ms_per_step'], d['roofline']['kernel_ms_per_tick'], d['exchange_csr_ms']))" | tee -a $OUT/ab.txt
  done
done
