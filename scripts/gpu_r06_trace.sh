#!/bin/bash
# round 6: rocprofv3 kernel trace + stats of the driver's bench command (N = 1, --steps 20
# --warmup 5), the per-kernel averages committed under profiles/r06/
cd "$GRAFT_REPO_ROOT" || exit 2
OUT="$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r06trace}"; mkdir -p "$OUT"
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp || exit 2
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
    python3 "$R/bench.py" --steps 20 --warmup 5 > "$OUT/bench20_traced.log" 2>&1 || exit $?
cp "$(ls "$OUT"/prof/*kernel_stats.csv | head -1)" "$OUT/kernel_stats_bench20.csv"
rm -f "$OUT"/prof/*kernel_trace.csv
echo done
