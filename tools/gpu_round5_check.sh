#!/bin/bash
# GPU parity suite, then configs 2 and 3 (no CPU baseline): the routine check after an engine change.
# usage: tools/gpu_round5_check.sh <outdir-under-gpurun_out> [pytest -k expr]
set -o pipefail
OUT=gpurun_out/${1:-check}; mkdir -p $OUT
export PYTHONUNBUFFERED=1
K=${2:+-k "$2"}
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread $K > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || { tail -40 $OUT/pytest.log; exit $rc; }
for c in config2 config3; do
  timeout -k 10 300 python -u bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline --no-ingest > $OUT/${c}.json 2> $OUT/${c}.err || { echo FAIL $c; tail -20 $OUT/${c}.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/${c}.json'));print('$c', round(d['value']/1e6,2), 'M ops/s', round(d['ms_per_step'],1), 'ms', d.get('parity'))"
done
