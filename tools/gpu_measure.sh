#!/bin/bash
# Measurement pass: bench lines with the CPU baseline and the widened oracle parity samples
# (config 4: all 256 documents; config 5: 4096 documents) and the snapshot times.
# usage: tools/gpu_measure.sh <outdir under gpurun_out> [configs...]
set -o pipefail
O=gpurun_out/${1:-r04m}; shift
CFGS=${@:-config3 config4 config5}
mkdir -p $O
export PYTHONUNBUFFERED=1
for c in $CFGS; do
  X=""; [ $c = config4 ] && X="--parity-docs 256"
  timeout -k 10 900 python -u bench.py --config $c $X > $O/${c}_bench.json 2> $O/${c}_bench.err || { echo FAIL $c; tail -20 $O/${c}_bench.err; exit 1; }
  python -c "import json;d=json.load(open('$O/${c}_bench.json'));print('$c', round(d['value']/1e6,2), 'M ops/s', round(d['ms_per_step'],1), 'ms/step', d['parity'], 'snapshot', d.get('snapshot',{}).get('ms'))"
done
