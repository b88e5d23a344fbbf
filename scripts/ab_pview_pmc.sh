#!/bin/bash
# GPU A/B of partial-view kernel variants on the driver's window (ticks 6-25): two timing runs
# per variant (interleaved), then one PMC pass per variant (instruction counts per tick over the
# same window, scripts/pmc_window.py).
#   bash scripts/ab_pview_pmc.sh <tag> <variant>...   ("base" = the product library)
cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
OUT="$GRAFT_REPO_ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for rep in 1 2; do
    for v in "$@"; do
        if [ "$v" = base ]; then VAR=""; else VAR="$v"; fi
        GSP_LIB_VARIANT=$VAR timeout -k 10 150 python3 -u scripts/bench_pview.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/$v-$rep.log" 2>&1
        rc=$?
        echo "$v rep$rep rc=$rc $(tail -1 "$OUT/$v-$rep.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("kernel_ms=%.3f csr_ms=%.3f ms_per_step=%.3f" % (d["roofline"]["kernel_ms_per_tick"], d["exchange_csr_ms"], d["ms_per_step"]))' 2>/dev/null)"
        [ $rc -ne 0 ] && exit $rc
    done
done
cd /tmp
for v in "$@"; do
    if [ "$v" = base ]; then VAR=""; else VAR="$v"; fi
    GSP_LIB_VARIANT=$VAR timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY -d "$OUT/pmc_$v" -o run --output-format csv -- python3 $R/scripts/bench_pview.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/pmc_$v.log" 2>&1
    rc=$?
    [ $rc -ne 0 ] && { echo "pmc $v rc=$rc"; exit $rc; }
    python3 $R/scripts/pmc_window.py $(ls "$OUT"/pmc_$v/*counter_collection.csv) --anchor pview_receipt_kernel --ticks 6 25 --kernels pview_tick --json "$OUT/pmc_$v.json" | python3 -c "
import json,sys; d=json.load(sys.stdin); print('$v', 'VALU/tick %.4g SALU/tick %.4g' % (d['SQ_INSTS_VALU']['per_tick'], d['SQ_INSTS_SALU']['per_tick']))"
done
echo done
