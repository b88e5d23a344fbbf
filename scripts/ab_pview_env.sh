cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab_q7
export TMPDIR=/tmp
run() { local name=$1; shift
  env "$@" timeout -k 10 150 python3 -u scripts/bench_pview.py --steps 10 --warmup 5 --no-cpu-baseline > gpurun_out/ab_q7/$name.log 2>&1 || exit 1
  echo "$name $(tail -1 gpurun_out/ab_q7/$name.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("kernel_ms=%.3f" % d["roofline"]["kernel_ms"])')"
}
run base1 GSP_PV_WAVES=8
run q7_1 GSP_LIB_VARIANT=q7
run w7_1 GSP_PV_WAVES=7
run base2 GSP_PV_WAVES=8
run q7_2 GSP_LIB_VARIANT=q7
run w7_2 GSP_PV_WAVES=7
echo done
