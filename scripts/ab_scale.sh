#!/bin/bash
# GPU A/B of full-view tick-kernel library variants at config 3: bash scripts/ab_scale.sh <tag> <variant>...
# ("base" = the product library; others = libgossip_amd.<variant>.so)
cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
OUT="$GRAFT_REPO_ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for v in "$@"; do
    if [ "$v" = base ]; then VAR=""; else VAR="$v"; fi
    i=$((i + 1))
    GSP_LIB_VARIANT=$VAR timeout -k 10 150 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-pview > "$OUT/$i-$v.log" 2>&1
    rc=$?
    echo "$v rc=$rc $(tail -1 "$OUT/$i-$v.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("kernel_ms=%.3f ms_per_step=%.3f" % (d["roofline"]["kernel_ms_per_tick"], d["ms_per_step"]))' 2>/dev/null)"
    [ $rc -ne 0 ] && exit $rc
done
echo done
