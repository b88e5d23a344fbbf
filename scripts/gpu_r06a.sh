#!/bin/bash
# round 6: drain-all hash classes -- parity first, then the drain bench and a phase profile
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r06a}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_pview_drain_gpu.py ${KSEL:+-k "$KSEL"} -x -v --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -5 $OUT/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u scripts/bench_pview.py --inbox 0 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/drain.json 2> $OUT/drain.err || exit 1
tail -c 1500 $OUT/drain.json
GSP_PV_PROFILE=1 timeout -k 10 300 python3 -u scripts/bench_pview.py --inbox 0 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/prof.json 2> $OUT/prof.log || exit 1
grep phases $OUT/prof.log
