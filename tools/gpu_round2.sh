#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python tools/phase_profile.py config2 4096 > gpurun_out/phase.log 2>&1 || { echo PHASE_FAIL; tail -20 gpurun_out/phase.log; exit 1; }
cat gpurun_out/phase.log
timeout -k 10 600 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { echo BENCH_FAIL; tail -20 gpurun_out/bench_default.err; exit 1; }
cat gpurun_out/bench_default.json
