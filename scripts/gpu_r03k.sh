#!/bin/bash
# Round 3: is the partial-view tick kernel bound by the CU's one scalar unit?  Lists the SQ
# counters this rocprofv3 offers, then one PMC pass (SALU / VALU instruction counts and cycles)
# over a short config-5 run; per split-kernel instance via scripts/pmc_by_kernel.py.
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r03k}
OUT="$GRAFT_REPO_ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 60 rocprofv3 --list-avail > "$OUT/avail.txt" 2>&1
echo "list rc=$?"
grep -o "SQ_[A-Z_]*\|GRBM_[A-Z_]*" "$OUT/avail.txt" | sort -u > "$OUT/sq_names.txt"
wc -l < "$OUT/sq_names.txt"
want=""
for c in SQ_INST_CYCLES_SALU SQ_INSTS_SALU SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_INST_CYCLES_VMEM; do
    grep -qx "$c" "$OUT/sq_names.txt" && want="$want $c"
done
echo "pass counters:$want GRBM_GUI_ACTIVE"
BENCH="$GRAFT_REPO_ROOT/scripts/bench_pview.py --steps 6 --warmup 4 --no-cpu-baseline"
timeout -s KILL 120 rocprofv3 --pmc $want GRBM_GUI_ACTIVE -d "$OUT/salu" -o run --output-format csv -- python3 $BENCH > "$OUT/salu.log" 2>&1
rc=$?
echo "salu rc=$rc"
[ $rc -ne 0 ] && exit $rc
cd "$GRAFT_REPO_ROOT"
python3 scripts/pmc_by_kernel.py pview_tick_split_kernel $(ls "$OUT"/salu/*counter_collection.csv) --json "$OUT/salu.json" > "$OUT/salu.txt"
cat "$OUT/salu.txt"
echo done
