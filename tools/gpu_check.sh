#!/bin/bash
# GPU parity + a short default bench (config 2): the round's routine check.
# usage: tools/gpu_check.sh <outdir-under-gpurun_out> [extra pytest -k expr]
set -o pipefail
OUT=gpurun_out/${1:-check}
mkdir -p $OUT
K=${2:+-k "$2"}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread $K > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
