#!/bin/bash
# phase profile of drain-all variants (GSP_PV_PROFILE=1): bash scripts/gpu_probe.sh <tag> <variant>...
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1; shift; mkdir -p $OUT
for v in "$@"; do
  if [ "$v" = base ]; then VAR=""; else VAR="$v"; fi
  GSP_LIB_VARIANT=$VAR GSP_PV_PROFILE=1 timeout -k 10 200 python3 -u scripts/bench_pview.py --inbox 0 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/$v.json 2> $OUT/$v.log || exit 1
  echo "== $v"; grep "k=8 \|k=9 " $OUT/$v.log
done
