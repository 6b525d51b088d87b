#!/bin/bash
# Config 5 with the wide block-residency size class at several thresholds (A/B against off),
# after the size-class parity tests.  usage: tools/gpu_c5_sizeclass.sh <outdir> [thresholds...]
set -o pipefail
OUT=gpurun_out/${1:-c5sc}; shift; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "size_class or long or config5" > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || { tail -30 $OUT/pytest.log; exit $rc; }
for t in "$@"; do
  timeout -k 10 400 python -u bench.py --config config5 --steps 3 --warmup 1 --no-cpu-baseline --no-ingest --big-min-ops $t > $OUT/c5_$t.json 2> $OUT/c5_$t.err || { echo FAIL $t; tail -20 $OUT/c5_$t.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/c5_$t.json'));print('big_min_ops', $t, round(d['value']/1e6,2), 'M ops/s', round(d['ms_per_step'],1), 'ms', d['parity'])"
done
