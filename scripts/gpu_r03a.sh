set -o pipefail
mkdir -p gpurun_out/r03b
timeout -k 10 120 python -c "import torch; f,t=torch.cuda.mem_get_info(); print('mem_get_info free', f, 'total', t)" > gpurun_out/r03b/mem.txt 2>&1 &&
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_scale_gpu.py -k "columns8 or config4" > gpurun_out/r03b/tests.log 2>&1 &&
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r03b/bench.json 2> gpurun_out/r03b/bench.err
