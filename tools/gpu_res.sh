#!/bin/bash
# Parity tests, then config2/config3 benches in each listed residency.
set -o pipefail
O=gpurun_out/res
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for cfg in ${CFGS:-config2 config3}; do
  for res in ${RES:-hbm blk}; do
    timeout -k 10 600 python bench.py --config $cfg --residency $res --no-cpu-baseline --steps 3 --warmup 1 > $O/$cfg.$res.json 2> $O/$cfg.$res.err || { echo BENCH_FAIL $cfg $res; tail -20 $O/$cfg.$res.err; exit 1; }
    python -c "import json;d=json.load(open('$O/$cfg.$res.json'));print('$cfg $res', round(d['value']/1e6,3),'Mops/s', round(d['roofline']['kernel_ms'],1),'ms', d['parity'])"
  done
done
