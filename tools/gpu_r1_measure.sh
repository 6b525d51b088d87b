#!/bin/bash
# Round-1 measurement pass: parity (pytest -m gpu, smoke), the default bench line,
# rocprofv3 kernel-trace stats of the bench, and HBM traffic PMC passes
# (FETCH_SIZE and WRITE_SIZE each in their own run, MI355X_MICROARCH.md §HBM).
set -o pipefail
O=gpurun_out/r1m
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/kt_bench.json 2> $O/kt.err || { echo KT_FAIL; tail -5 $O/kt.err; exit 1; }
cat $O/kt_bench.json
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmcF -o pmcF -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/pmcF.json 2> $O/pmcF.err || { echo PMCF_FAIL; tail -5 $O/pmcF.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmcW -o pmcW -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/pmcW.json 2> $O/pmcW.err || { echo PMCW_FAIL; tail -5 $O/pmcW.err; exit 1; }
find $O -name "*.csv" | sort
