#!/bin/bash
# A/B of replay residency (LDS vs HBM pools) at two document counts + parity.
set -o pipefail
O=gpurun_out/ab
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for args in "--residency hbm" "--residency lds" "--residency hbm --docs 1536" "--residency lds --docs 1536" "--residency lds --docs 1536 --ops 3000" "--residency hbm --docs 1536 --ops 3000"; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 2 --warmup 1 $args > $O/b.json 2> $O/b.err || { echo BENCH_FAIL $args; tail -20 $O/b.err; exit 1; }
  python -c "import json;d=json.load(open('$O/b.json'));print('$args', round(d['value']/1e6,2),'Mops/s', round(d['roofline']['kernel_ms'],1),'ms')"
done
