#!/bin/bash
# Parity tests, then one bench line per listed config (no CPU baseline).
set -o pipefail
O=gpurun_out/m
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for cfg in ${CFGS:-config2 config4}; do
  timeout -k 10 600 python bench.py --config $cfg --no-cpu-baseline --steps ${STEPS:-3} --warmup 1 > $O/$cfg.json 2> $O/$cfg.err || { echo BENCH_FAIL $cfg; tail -20 $O/$cfg.err; exit 1; }
  python -c "import json;d=json.load(open('$O/$cfg.json'));print('$cfg', round(d['value']/1e6,3),'Mops/s', round(d['roofline']['kernel_ms'],1),'ms', d['parity'])"
done
