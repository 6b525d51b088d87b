#!/bin/bash
# Block-residency continuation classes (mt_set_continuation): configs 3 and 5 at several
# thresholds (0: every run keeps the in-wave continuation).  usage: tools/gpu_cont_ab.sh <outdir>
set -o pipefail
OUT=gpurun_out/${1:-cont}; mkdir -p $OUT
export PYTHONUNBUFFERED=1
for v in "config5 0" "config5 8192" "config5 16384" "config3 0" "config3 8192" "config2 0" "config2 16384"; do
  set -- $v
  timeout -k 10 400 python -u bench.py --config $1 --steps 3 --warmup 1 --no-cpu-baseline --no-ingest --cont-min $2 > $OUT/$1_$2.json 2> $OUT/$1_$2.err || { echo FAIL $v; tail -5 $OUT/$1_$2.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/$1_$2.json'));print('$1 cont-min $2', round(d['value']/1e6,2), 'M ops/s', round(d['ms_per_step'],1), 'ms', d['parity'])"
done
