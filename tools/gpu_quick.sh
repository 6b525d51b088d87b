#!/bin/bash
# Quick GPU pass: parity tests, smoke, one bench line (no CPU baseline), kernel stats.
set -o pipefail
O=gpurun_out/q
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > $O/kt_bench.json 2> $O/kt.err || { echo KT_FAIL; tail -5 $O/kt.err; exit 1; }
cat $O/kt/kt_kernel_stats.csv
