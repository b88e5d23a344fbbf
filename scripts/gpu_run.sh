#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
nproc; rocm-smi --showproductname 2>/dev/null | head -5
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r1_tests.log 2>&1
rc=$?
echo "tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 240 python -u bench.py > gpurun_out/r1_bench.json 2> gpurun_out/r1_bench.err
rc=$?
echo "bench rc=$rc"; cat gpurun_out/r1_bench.json
if [ $rc -ne 0 ]; then exit $rc; fi
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof1" -o bench --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 5 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/r1_prof.log" 2>&1
echo "prof rc=$?"
