#!/bin/bash
# round 6: the -m gpu suite in two halves (PART=a: everything but the partial-view files; PART=b:
# the partial-view and drain-all files), each under its own limit
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r06suite}; mkdir -p $OUT
if [ "${PART:-a}" = a ]; then SEL="--ignore=tests/test_pview_gpu.py --ignore=tests/test_pview_drain_gpu.py"; else SEL="tests/test_pview_gpu.py tests/test_pview_drain_gpu.py"; fi
[ "${PART:-a}" = a ] && T=tests || T=
timeout -k 10 1080 python -u -m pytest $T $SEL -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests_${PART:-a}.log 2>&1
rc=$?; tail -3 $OUT/tests_${PART:-a}.log; exit $rc
