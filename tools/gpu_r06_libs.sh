#!/bin/bash
# Engine-library A/B on one box, alternating, partition off (same kernels for every library).
# usage: CFGS="config2" ROUNDS=2 tools/gpu_r06_libs.sh <outdir> <lib.so>...
set -o pipefail
O=gpurun_out/${1:-r06_libs}; shift; mkdir -p $O
export PYTHONUNBUFFERED=1
for r in $(seq 1 ${ROUNDS:-2}); do
  for lib in "$@"; do
    for c in ${CFGS:-config2}; do
      n=$(basename $lib .so)_${c}_$r
      MTGPU_LIB=$lib timeout -k 10 300 python -u bench.py --config $c ${OPS:+--ops $OPS} --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline --no-ingest --partition off > $O/$n.json 2> $O/$n.err || { echo FAIL $n; tail -20 $O/$n.err; exit 1; }
      python -c "import json;d=json.load(open('$O/$n.json'));print('$n', round(d['value']/1e6,2), 'M ops/s', round(d['ms_per_step'],1), 'ms', d['parity'][-24:])"
    done
  done
done
