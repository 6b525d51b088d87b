#!/bin/bash
# Bench lines for a set of configs (no CPU baseline, no ingest): a quick A/B of a kernel change.
# usage: tools/gpu_bench_set.sh <outdir-under-gpurun_out> [configs...]
set -o pipefail
OUT=gpurun_out/${1:-set}; shift
CFGS=${@:-config2 config4 config5}
mkdir -p $OUT
export PYTHONUNBUFFERED=1
for c in $CFGS; do
  timeout -k 10 400 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-ingest > $OUT/${c}.json 2> $OUT/${c}.err || { echo FAIL $c; tail -20 $OUT/${c}.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/${c}.json'));print('$c', round(d['value']/1e6,2), 'M ops/s', round(d['roofline']['kernel_ms'],1), 'ms', d['parity'])"
done
