#!/bin/bash
# GPU session: partial-view library variants side by side -- phase profile (GSP_PV_PROFILE)
# and one SQ instruction-count PMC pass each.
# usage: bash scripts/gpu_pv_cmp.sh <tag> <variant>...   ("base" = the product library)
set -uo pipefail
: "${GRAFT_REPO_ROOT:?run on the GPU box (gpurun exports GRAFT_REPO_ROOT)}"
if [ $# -lt 2 ]; then
    echo "usage: $0 <tag> <variant>..." >&2
    exit 2
fi
cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
OUT="$GRAFT_REPO_ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in "$@"; do
    if [ "$v" = base ]; then VAR=""; else VAR="$v"; fi
    timeout -k 10 200 env GSP_LIB_VARIANT=$VAR GSP_PV_PROFILE=1 python3 -u scripts/bench_pview.py \
        --steps 10 --warmup 5 --no-cpu-baseline > "$OUT/phases_$v.log" 2>&1
    rc=$?; echo "$v phases rc=$rc"; [ $rc -ne 0 ] && exit $rc
    grep "pview phases" "$OUT/phases_$v.log" | tail -1
    (cd /tmp && timeout -k 10 120 env GSP_LIB_VARIANT=$VAR rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU \
        SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
        -d "$OUT/pmc_$v" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/scripts/bench_pview.py" \
        --steps 3 --warmup 5 --no-cpu-baseline > "$OUT/pmc_$v.log" 2>&1)
    rc=$?; echo "$v pmc rc=$rc"; [ $rc -ne 0 ] && exit $rc
    python3 scripts/pmc_summary.py "pview_tick_kernel<8, 0>" "$OUT/pmc_$v/run_counter_collection.csv" \
        --json "$OUT/summary_$v.json"
done
echo done
