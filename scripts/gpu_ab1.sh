#!/bin/bash
# partial-view parity suites, then an environment A/B of the tick kernel (scripts/ab_pview_env.sh)
#   bash scripts/gpu_ab1.sh <tag> <name>:<ENV=V>[,...] ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:?usage: $0 <tag> <specs>...}; shift
mkdir -p "gpurun_out/$TAG"
timeout -k 10 500 python -u -m pytest tests/test_pview_gpu.py tests/test_events_gpu.py tests/test_policy_gpu.py -x -q \
    --timeout 200 --timeout-method thread > "gpurun_out/$TAG/tests.log" 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 "gpurun_out/$TAG/tests.log"
[ $rc -ne 0 ] && exit $rc
bash scripts/ab_pview_env.sh "$TAG" "$@"
