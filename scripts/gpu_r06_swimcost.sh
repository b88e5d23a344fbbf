#!/bin/bash
# round 6: where the SWIM + TFAIL drained run's extra kernel time goes -- rocprofv3 kernel stats
# of config 5 drained, plain (removal records on) and with swim = 2, tfail = 5
cd "$GRAFT_REPO_ROOT" || exit 2
OUT="$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r06sw}"; mkdir -p "$OUT"
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp || exit 2
for v in plain swim tfail both; do
  case $v in plain) S=0; T=0;; swim) S=2; T=0;; tfail) S=0; T=5;; both) S=2; T=5;; esac
  PV_SWIM=$S PV_TFAIL=$T PV_EVENTS=4 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/$v" -o run --output-format csv -- \
      python3 "$R/scripts/pv_variant_trace.py" > "$OUT/$v.log" 2>&1 || exit $?
  rm -f "$OUT"/$v/*kernel_trace.csv
  grep kernel_ms "$OUT/$v.log"
done
