#!/bin/bash
# A/B: committed engine (base) vs current (W=4) vs W=3, plus rocprofv3 kernel stats.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for v in base w3; do
  MTGPU_LIB=$PWD/fluidframework_amd/libmtgpu_$v.so timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_$v.json 2> gpurun_out/bench_$v.err || { echo BENCH_${v}_FAIL; tail -20 gpurun_out/bench_$v.err; exit 1; }
  cat gpurun_out/bench_$v.json
done
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { echo BENCH_FAIL; tail -20 gpurun_out/bench_default.err; exit 1; }
cat gpurun_out/bench_default.json
timeout -k 10 300 python tools/phase_profile.py config2 4096 > gpurun_out/phase.log 2>&1 || { echo PHASE_FAIL; tail -20 gpurun_out/phase.log; exit 1; }
cat gpurun_out/phase.log
