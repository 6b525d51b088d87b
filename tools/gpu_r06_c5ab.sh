#!/bin/bash
# Config-5 library A/B at bench's default (automatic partition), alternating rounds.
# usage: ROUNDS=2 tools/gpu_r06_c5ab.sh <outdir> <lib.so>...
set -o pipefail
O=gpurun_out/${1:-r06_c5ab}; shift; mkdir -p $O
export PYTHONUNBUFFERED=1
for r in $(seq 1 ${ROUNDS:-2}); do
  for lib in "$@"; do
    n=$(basename $lib .so)_c5_$r
    MTGPU_LIB=$lib timeout -k 10 400 python -u bench.py --config config5 --steps 3 --warmup 1 --no-cpu-baseline > $O/$n.json 2> $O/$n.err || { echo FAIL $n; tail -20 $O/$n.err; exit 1; }
    python -c "import json;d=json.load(open('$O/$n.json'));print('$n', round(d['value']/1e6,2), 'M ops/s', round(d['ms_per_step'],1), 'ms', d['config'].get('partition'), d['parity'][-24:])"
  done
done
