#!/bin/bash
# GPU validation + first measurements (run via gpurun from the repo root).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 120 python tools/probe_torch_coexist.py > gpurun_out/probe.log 2>&1; echo "probe rc=$?"; tail -3 gpurun_out/probe.log
timeout -k 10 300 python bench.py --docs 512 --ops 2000 --steps 2 --warmup 1 --cpu-seconds 5 > gpurun_out/bench_small.json 2> gpurun_out/bench_small.err || { echo BENCH_SMALL_FAIL; tail -20 gpurun_out/bench_small.err; exit 1; }
cat gpurun_out/bench_small.json
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { echo BENCH_FAIL; tail -20 gpurun_out/bench_default.err; exit 1; }
cat gpurun_out/bench_default.json
