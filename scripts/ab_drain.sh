#!/bin/bash
# Drain-all (inbox 0) A/B of library variants: two interleaved runs of scripts/bench_pview.py
# --inbox 0 (ticks 6-25, the driver's window) per variant ("base" = the product library, others
# GSP_LIB_VARIANT); prints each run's tick-kernel ms and the drain classes' ms.
#   bash scripts/ab_drain.sh <tag> base <variant>...
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1; shift; mkdir -p $OUT
for rep in 1 2; do for v in "$@"; do
  if [ "$v" = base ]; then VAR=""; else VAR="$v"; fi
  GSP_LIB_VARIANT=$VAR timeout -k 10 200 python3 -u scripts/bench_pview.py --inbox 0 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/$v-$rep.log 2>&1 || exit 1
  python3 - $OUT/$v-$rep.log $v $rep <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
dc = d.get("drain_classes", [])
print("%-12s rep%s tick-kernels %.3f ms  drain %.3f ms  [%s]" % (sys.argv[2], sys.argv[3], d["roofline"]["kernel_ms_per_tick"],
      sum(c["kernel_ms_per_tick"] for c in dc), " ".join("%.3f" % c["kernel_ms_per_tick"] for c in dc)))
PY
done; done
