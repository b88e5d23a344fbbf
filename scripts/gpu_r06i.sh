#!/bin/bash
# round 6: drain parity (LDS classes, events, extensions),
# then the drain bench and a phase profile
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r06i}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_pview_drain_gpu.py -k "${KSEL:-not full_size}" -x -v --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -4 $OUT/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u scripts/bench_pview.py --inbox 0 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/drain.json 2> $OUT/drain.err || exit 1
python3 - $OUT/drain.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
dc = d.get("drain_classes", [])
print("tick-kernels %.3f ms  drain %.3f ms  [%s]" % (d["roofline"]["kernel_ms_per_tick"], sum(c["kernel_ms_per_tick"] for c in dc), " ".join("%.3f" % c["kernel_ms_per_tick"] for c in dc)))
PY
GSP_PV_PROFILE=1 timeout -k 10 300 python3 -u scripts/bench_pview.py --inbox 0 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/prof.json 2> $OUT/prof.log || exit 1
grep "k=8\|k=9\|k=1[0-5]" $OUT/prof.log
