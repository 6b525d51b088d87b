#!/bin/bash
# Round 4: A/B of the no-newline row flag (MT_NONL=0 build vs the product), then the round-4
# measurement lines (configs 3, 4, 5 with CPU baseline and widened parity samples).
set -o pipefail
OUT=gpurun_out/r04_nonl; mkdir -p $OUT
export PYTHONUNBUFFERED=1
for c in config2 config3 config5; do
  for v in nonl0 product; do
    L=fluidframework_amd/libmtgpu.so; [ $v = nonl0 ] && L=fluidframework_amd/libmtgpu_nonl0.so
    MTGPU_LIB=$L timeout -k 10 400 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-ingest > $OUT/${c}_$v.json 2> $OUT/${c}_$v.err || { echo FAIL $c $v; tail -5 $OUT/${c}_$v.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/${c}_$v.json'));print('$c $v', round(d['value']/1e6,2), 'M ops/s', round(d['roofline']['kernel_ms'],1), 'ms', d['parity'])"
  done
done
bash tools/gpu_r04_measure.sh r04m config3 config4 config5
