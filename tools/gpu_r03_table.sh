#!/bin/bash
# Round 3: long documents (corrections table, block cache, zamboni prefetch) -- long-document
# GPU parity, config 4 with the switches (MT_BIGF_*) on and off, config 2 check.
set -o pipefail
OUT=gpurun_out/r03_tab; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_long_docs.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for f in 0 1 2 4 7; do
  timeout -k 10 400 python -u bench.py --config config4 --steps 2 --warmup 1 --no-cpu-baseline --no-ingest --big-flags $f > $OUT/c4_f$f.json 2> $OUT/c4_f$f.err || { echo FAIL $f; tail -20 $OUT/c4_f$f.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/c4_f$f.json'));print('config4 big-flags $f', round(d['value']/1e6,3), 'M ops/s', round(d['roofline']['kernel_ms'],1), 'ms', d['parity'])"
done
timeout -k 10 400 python -u bench.py --config config2 --steps 3 --warmup 1 --no-cpu-baseline --no-ingest > $OUT/c2.json 2> $OUT/c2.err || { echo FAIL c2; tail -20 $OUT/c2.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/c2.json'));print('config2', round(d['value']/1e6,3), 'M ops/s', round(d['roofline']['kernel_ms'],1), 'ms', d['parity'])"
