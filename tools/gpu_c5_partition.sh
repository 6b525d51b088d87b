#!/bin/bash
# Config 5 with partitioned size classes (long runs in the wide block-residency kernel on
# reserved CUs): A/B over MIN:CUS specs.  usage: tools/gpu_c5_partition.sh <outdir> <spec...>
set -o pipefail
OUT=gpurun_out/${1:-c5part}; shift; mkdir -p $OUT
export PYTHONUNBUFFERED=1
for t in "$@"; do
  n=${t/:/_}
  timeout -k 10 400 python -u bench.py --config config5 --steps 3 --warmup 1 --no-cpu-baseline --no-ingest --partition $t > $OUT/c5_$n.json 2> $OUT/c5_$n.err || { echo FAIL $t; tail -20 $OUT/c5_$n.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/c5_$n.json'));print('partition', '$t', round(d['value']/1e6,2), 'M ops/s', round(d['ms_per_step'],1), 'ms', d['parity'][-40:])"
done
