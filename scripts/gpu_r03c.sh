#!/bin/bash
# Round 3 profiling session: counters of every partial-view split kernel instance
#  and L2 hit / miss per full-view tile launch at G = 1/4/8/16 (item 5).
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r03c}
OUT="$GRAFT_REPO_ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {   # step <name> <timeout> cmd...; stop the session on a crash / timeout
    local name=$1 to=$2; shift 2
    timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"
    if [ $rc -ne 0 ]; then exit $rc; fi
}
step avail 60 rocprofv3 -L
cd /tmp
PVB="$GRAFT_REPO_ROOT/scripts/bench_pview.py --steps 10 --warmup 5 --no-cpu-baseline"
step pv_sq1 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS -d "$OUT/pv_sq1" -o run --output-format csv -- python3 $PVB
step pv_sq2 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA -d "$OUT/pv_sq2" -o run --output-format csv -- python3 $PVB
for G in 1 4 8 16; do
    step tcc_g$G 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d "$OUT/tcc_g$G" -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/tile_run.py $G
done
step tcc_c4_32 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d "$OUT/tcc_c4_32" -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/tile_run.py 32 --nodes 262144 --ticks 3 --warmup 2
cd "$GRAFT_REPO_ROOT"
python3 scripts/pmc_by_kernel.py pview_tick_split_kernel $(ls "$OUT"/pv_sq*/*counter_collection.csv) --json "$OUT/pv_by_kernel.json" > "$OUT/pv_by_kernel.txt"
for G in 1 4 8 16; do
    python3 scripts/pmc_by_kernel.py scale_tick_kernel $(ls "$OUT"/tcc_g$G/*counter_collection.csv) --json "$OUT/tcc_g$G.json" > "$OUT/tcc_g$G.txt"
done
python3 scripts/pmc_by_kernel.py scale_tick_kernel $(ls "$OUT"/tcc_c4_32/*counter_collection.csv) --json "$OUT/tcc_c4_32.json" > "$OUT/tcc_c4_32.txt"
echo done
