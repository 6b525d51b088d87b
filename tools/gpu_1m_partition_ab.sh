#!/bin/bash
# north_star's 1,048,576-document config-5 line on one GPU, A/B over partition specs in one lease
# (review item r05-1).  usage: tools/gpu_1m_partition_ab.sh <outdir> <spec...>   (spec: off | MIN:CUS | auto)
set -o pipefail
OUT=gpurun_out/${1:-r06_1m_ab}; shift; mkdir -p $OUT
export PYTHONUNBUFFERED=1
for t in "$@"; do
  n=${t/:/_}
  timeout -k 10 420 python -u bench.py --config config5 --docs 1048576 --steps 2 --warmup 1 --no-cpu-baseline \
      --partition $t > $OUT/c5_1m_$n.json 2> $OUT/c5_1m_$n.err || { echo FAIL $t; tail -20 $OUT/c5_1m_$n.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/c5_1m_$n.json'));print('partition', '$t', round(d['value']/1e6,2), 'M ops/s', round(d['ms_per_step'],1), 'ms', d['config']['partition'], d['parity'][-60:])"
done
