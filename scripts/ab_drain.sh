#!/bin/bash
# Drain-all (inbox 0) A/B of library variants: two interleaved runs of scripts/bench_pview.py
# --inbox 0 (ticks 6-35) per variant ("base" = the product library, others GSP_LIB_VARIANT).
#   bash scripts/ab_drain.sh <tag> base <variant>...
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1; shift; mkdir -p $OUT
for rep in 1 2; do for v in "$@"; do
  if [ "$v" = base ]; then VAR=""; else VAR="$v"; fi
  GSP_LIB_VARIANT=$VAR timeout -k 10 200 python3 -u scripts/bench_pview.py --inbox 0 --steps 30 --warmup 5 --no-cpu-baseline > $OUT/$v-$rep.log 2>&1 || exit 1
  echo "$v rep$rep $(grep -o '"ms_per_step": [0-9.]*' $OUT/$v-$rep.log | head -1)"
done; done
