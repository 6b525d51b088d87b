#!/bin/bash
# Round 4 pass 7: the GPU suite, then configs 2-5 (window entries and leaf lengths read as row quads; the
# direct-mapped parent cache back; snapshot staging groups in whole thread rounds).
set -o pipefail
OUT=gpurun_out/${OUTDIR:-r04_ab7}; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $OUT/gpu_suite.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -2 $OUT/gpu_suite.log; [ $rc -eq 0 ] || exit $rc
for c in config2 config3 config4 config5; do
  timeout -k 10 500 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-ingest > $OUT/${c}.json 2> $OUT/${c}.err || { echo FAIL $c; tail -5 $OUT/${c}.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/${c}.json'));print('$c', round(d['value']/1e6,2), 'M ops/s', round(d['roofline']['kernel_ms'],1), 'ms', d['parity'], 'snapshot', round(d.get('snapshot',{}).get('ms',0),1))"
done
