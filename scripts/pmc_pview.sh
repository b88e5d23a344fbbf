#!/bin/bash
# PMC passes of the partial-view tick kernels over the driver's window (ticks 6-25), one
# rocprofv3 pass per counter group (SQ issue counters, FETCH_SIZE, WRITE_SIZE), each under its
# own time limit; scripts/pmc_pview_json.py turns them into profiles/pmc_sq_pview.json and
# profiles/pmc_traffic_pview.json (drain all, INBOX=0, the default) or the _inbox7 files
# (INBOX=7) -- what bench.py reads when its window matches.
#   [INBOX=7] bash scripts/pmc_pview.sh <tag>
cd "$GRAFT_REPO_ROOT" || exit 2
TAG=${1:?usage: $0 <tag>}
OUT="$GRAFT_REPO_ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp || exit 2
pass() {   # pass <name> <counters...>
    local name=$1; shift
    timeout -k 10 240 rocprofv3 --pmc "$@" -d "$OUT/pmc_$name" -o run --output-format csv -- \
        python3 "$R/scripts/bench_pview.py" --steps 20 --warmup 5 --no-cpu-baseline --inbox ${INBOX:-0} > "$OUT/pmc_$name.log" 2>&1
    local rc=$?
    echo "pmc $name rc=$rc"
    [ $rc -eq 0 ] || exit $rc
}
pass sq SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU
pass fetch FETCH_SIZE
pass write WRITE_SIZE
python3 "$R/scripts/pmc_pview_json.py" "$OUT" --inbox ${INBOX:-0} && echo done
