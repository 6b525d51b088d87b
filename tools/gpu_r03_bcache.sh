#!/bin/bash
# Round 3: LDS block cache for long documents -- long-document GPU parity, then config 4
# (and config 5) with the cache on and off.
set -o pipefail
OUT=gpurun_out/r03_bc; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_long_docs.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for v in on off; do
  f=""; [ $v = off ] && f="--no-bcache"
  timeout -k 10 400 python -u bench.py --config config4 --steps 2 --warmup 1 --no-cpu-baseline --no-ingest $f > $OUT/c4_$v.json 2> $OUT/c4_$v.err || { echo FAIL $v; tail -20 $OUT/c4_$v.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/c4_$v.json'));print('config4 bcache $v', round(d['value']/1e6,3), 'M ops/s', round(d['roofline']['kernel_ms'],1), 'ms', d['parity'])"
done
timeout -k 10 300 python -u tools/phase_config4.py 256 200000 5000 big > $OUT/phase_c4_big.log 2>&1 || { tail -20 $OUT/phase_c4_big.log; exit 1; }
cat $OUT/phase_c4_big.log
