#!/bin/bash
# Round 3: partial-view parity of the launch forms, A/B of the kernel forms / library variants
# (AB="name:ENV=val ..."; GSP_LIB_VARIANT=<tag> loads libgossip_amd.<tag>.so), and a per-k
# phase profile (GSP_PV_PROFILE=1).
#   bash scripts/gpu_r03h.sh <tag>
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r03h}
OUT="$GRAFT_REPO_ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {   # step <name> <timeout> cmd...; stop the session on a failure / crash / timeout
    local name=$1 to=$2; shift 2
    timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"
    if [ $rc -ne 0 ]; then exit $rc; fi
}
if [ "${SKIP_TESTS:-0}" = 0 ]; then
    step tests 900 python -u -m pytest ${TESTS:-tests/test_pview_gpu.py} -m gpu -x -v --timeout 300 --timeout-method thread
    tail -1 "$OUT/tests.log"
fi
for v in ${VARIANTS:-}; do     # library variants: parity of the launch forms first
    step parity_$v 400 env GSP_LIB_VARIANT=$v python -u -m pytest ${VARIANT_TESTS:-tests/test_pview_gpu.py} -x -q --timeout 120 --timeout-method thread -k "${PARITY_K:-kernel_forms or full_size}"
    tail -1 "$OUT/parity_$v.log"
done
for i in 1 2; do
    for spec in ${AB:-base: exact:GSP_PV_SPLITSYNC=1}; do
        name=${spec%%:*}
        envs=${spec#*:}
        envs=${envs//,/ }              # several settings: NAME=a,OTHER=b
        step ab_${name}_$i 150 env $envs python3 -u scripts/bench_pview.py --steps 20 --warmup 5 --no-cpu-baseline
        echo "$name $i $(tail -1 "$OUT/ab_${name}_$i.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("kernel_ms=%.3f csr_ms=%.3f step_ms=%.3f" % (d["roofline"]["kernel_ms_per_tick"], d["exchange_csr_ms"], d["ms_per_step"]))')"
    done
done
if [ "${PROF:-1}" = 1 ]; then
    step pvprof 150 env GSP_PV_PROFILE=1 ${PROF_ENV:-} python3 -u scripts/bench_pview.py --steps 20 --warmup 5 --no-cpu-baseline
    grep "pview phases" "$OUT/pvprof.log"
fi
echo done
