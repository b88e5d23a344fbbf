#!/bin/bash
# One PMC pass of the partial-view tick kernels' LDS counters over the driver's window
# (ticks 6-25): LDS instructions, LDS-array busy cycles and bank-conflict cycles.
#   bash scripts/pmc_pview_lds.sh <tag>
cd "$GRAFT_REPO_ROOT" || exit 2
TAG=${1:?usage: $0 <tag>}
OUT="$GRAFT_REPO_ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp || exit 2
timeout -k 10 240 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU \
    -d "$OUT/pmc_lds" -o run --output-format csv -- python3 "$R/scripts/bench_pview.py" --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/pmc_lds.log" 2>&1
rc=$?
echo "pmc lds rc=$rc"
[ $rc -eq 0 ] || exit $rc
python3 "$R/scripts/pmc_window.py" $(ls "$OUT"/pmc_lds/*counter_collection.csv) --anchor pview_receipt_kernel --ticks 6 25 --kernels pview_tick --json "$OUT/pmc_lds.json" > /dev/null && python3 - "$OUT/pmc_lds.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))["counters"]
for k, v in sorted(d.items()):
    print(k, "%.4g per tick" % v["per_tick"])
PY
echo done
