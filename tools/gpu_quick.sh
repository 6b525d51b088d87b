#!/bin/bash
# Quick GPU pass: parity tests, config-2 bench (no CPU baseline), optional extra command.
# usage: tools/gpu_quick.sh <outdir-under-gpurun_out> [pytest -k expr]
set -o pipefail
OUT=gpurun_out/${1:-quick}
mkdir -p $OUT
export PYTHONUNBUFFERED=1
K=${2:+-k "$2"}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread $K > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-ingest > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));print('config2', round(d['value']/1e6,2), 'M ops/s', d['ms_per_step'], d['parity'])"
