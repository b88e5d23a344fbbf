#!/bin/bash
# GPU session: PMC passes over a short partial-view bench (one rocprofv3 run per counter group)
cd "$GRAFT_REPO_ROOT"
TAG=${1:-pvpmc}
OUT="$GRAFT_REPO_ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
BENCH="$GRAFT_REPO_ROOT/scripts/bench_pview.py --steps 3 --warmup 2 --no-cpu-baseline"
cd /tmp
pass() {
    local name=$1; shift
    timeout -k 10 120 rocprofv3 --pmc "$@" -d "$OUT/$name" -o run --output-format csv -- python3 $BENCH > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"
    if [ $rc -ne 0 ]; then exit $rc; fi
}
pass sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS
pass sq2 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA
pass fetch FETCH_SIZE
pass write WRITE_SIZE
cd "$GRAFT_REPO_ROOT"
python3 scripts/pmc_summary.py "pview_tick_kernel<8, 0>" $(ls "$OUT"/*/run_counter_collection.csv) --json "$OUT/summary.json"
echo done
