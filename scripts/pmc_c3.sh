#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes of config 3's tick kernel (8 column tiles) over the driver's
# window (ticks 6-25 of bench.py --steps 20 --warmup 5, config 3 alone, event stream on as the
# headline runs it), one rocprofv3 pass per
# counter, each under its own time limit; scripts/pmc_c3_json.py writes profiles/pmc_traffic.json.
#   bash scripts/pmc_c3.sh <tag>
cd "$GRAFT_REPO_ROOT" || exit 2
TAG=${1:?usage: $0 <tag>}
OUT="$GRAFT_REPO_ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp || exit 2
for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 240 rocprofv3 --pmc $c -d "$OUT/pmc_c3_$c" -o run --output-format csv -- \
        python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-pview --no-262k --no-events-off \
        > "$OUT/pmc_c3_$c.log" 2>&1
    rc=$?
    echo "pmc $c rc=$rc"
    [ $rc -eq 0 ] || exit $rc
done
python3 "$R/scripts/pmc_c3_json.py" "$OUT" && echo done
