#!/bin/bash
# GPU A/B of partial-view runs that differ by environment (GSP_LIB_VARIANT=<tag> for a
# `make lib-variant` library, GSP_PV_WAVES=7|8, ...), interleaved as given:
#   bash scripts/ab_pview_env.sh <tag> base:GSP_PV_WAVES=8 w7:GSP_PV_WAVES=7 base2:GSP_PV_WAVES=8
# STEPS / WARMUP (environment, default 20 / 5: the driver's window, ticks 6-25) and EXTRA
# (more bench_pview.py arguments, e.g. "--inbox 0") apply to every run.
set -euo pipefail
: "${GRAFT_REPO_ROOT:?run on the GPU box (gpurun exports GRAFT_REPO_ROOT)}"
if [ $# -lt 2 ]; then
    echo "usage: $0 <tag> <name>:<ENV=V>[,<ENV=V>...] ..." >&2
    exit 2
fi
cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
OUT="$GRAFT_REPO_ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
for spec in "$@"; do
    name=${spec%%:*}
    IFS=, read -r -a envs <<< "${spec#*:}"
    env "${envs[@]}" timeout -k 10 150 python3 -u scripts/bench_pview.py --steps "${STEPS:-20}" \
        --warmup "${WARMUP:-5}" --no-cpu-baseline ${EXTRA:-} > "$OUT/$name.log" 2>&1
    echo "$name $(tail -1 "$OUT/$name.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("kernel_ms=%.3f csr_ms=%.3f step_ms=%.3f" % (d["roofline"]["kernel_ms_per_tick"], d["exchange_csr_ms"], d["ms_per_step"]))')"
done
echo done
