#!/bin/bash
# One GPU session: tests, bench, policy A/B, rocprof kernel trace + PMC passes.
# usage: bash scripts/gpu_run.sh <tag>
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r}
OUT="$GRAFT_REPO_ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {   # step <name> <timeout> cmd...; stop the session on a crash / timeout
    local name=$1 to=$2; shift 2
    timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
    return 0
}
step tests 420 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
step bench 240 python -u bench.py
cat "$OUT/bench.log" | tail -1
# step ab 200 python -u scripts/ab_policy.py 65536 4
# tail -1 "$OUT/ab.log"
cd /tmp
BENCH="$GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 5 --no-cpu-baseline --no-pview"
step prof_trace 200 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline
step pmc_fetch 120 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run --output-format csv -- python3 $BENCH
step pmc_write 120 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run --output-format csv -- python3 $BENCH
step pmc_sq 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d "$OUT/pmc_sq" -o run --output-format csv -- python3 $BENCH
step pmc_tcc 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d "$OUT/pmc_tcc" -o run --output-format csv -- python3 $BENCH
PVB="$GRAFT_REPO_ROOT/scripts/bench_pview.py --steps 30 --warmup 5 --no-cpu-baseline"
step pv_fetch 200 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pv_fetch" -o run --output-format csv -- python3 $PVB
step pv_write 200 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pv_write" -o run --output-format csv -- python3 $PVB
step pv_sq 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS -d "$OUT/pv_sq" -o run --output-format csv -- python3 $PVB
cd "$GRAFT_REPO_ROOT"
python3 scripts/pmc_traffic.py $(ls "$OUT"/pmc_fetch/*counter_collection.csv) $(ls "$OUT"/pmc_write/*counter_collection.csv) "$OUT/pmc_traffic.json" --tiles 8
python3 scripts/pmc_traffic.py $(ls "$OUT"/pv_fetch/*counter_collection.csv) $(ls "$OUT"/pv_write/*counter_collection.csv) "$OUT/pmc_traffic_pview.json" --pview
python3 scripts/pmc_summary.py "pview_tick_split_kernel<0, " $(ls "$OUT"/pv_sq/*counter_collection.csv) \
    --per-tick "pview_tick_split_kernel<0, 128, 0, 3," --json "$OUT/pmc_sq_pview.json"
echo done
