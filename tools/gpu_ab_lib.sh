#!/bin/bash
# A/B of two engine builds on bench configs: the product libmtgpu.so vs $ALT (MTGPU_LIB).
# usage: tools/gpu_ab_lib.sh <outdir> <alt-lib> <configs...>   (PYTEST=1: GPU parity suite first)
set -o pipefail
OUT=gpurun_out/$1; ALT=$2; shift 2
mkdir -p $OUT
export PYTHONUNBUFFERED=1
if [ -n "$PYTEST" ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
  tail -1 $OUT/pytest.log
fi
for c in "$@"; do
  for v in prod alt; do
    L=""; [ $v = alt ] && L=$ALT
    MTGPU_LIB=$L timeout -k 10 300 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-ingest > $OUT/${c}_$v.json 2> $OUT/${c}_$v.err || { echo FAIL $c $v; tail -20 $OUT/${c}_$v.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/${c}_$v.json'));print('$c $v', round(d['value']/1e6,3), 'M ops/s', round(d['roofline']['kernel_ms'],1), 'ms', d.get('parity'))"
  done
done
