#!/bin/bash
# Round-end check on one MI355X: the whole GPU suite, smoke(), the default bench line (as the
# driver runs it) and configs 3-5 without the CPU baseline.  usage: tools/gpu_final.sh <outdir>
set -o pipefail
OUT=gpurun_out/${1:-final}; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $OUT/gpu_suite.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -2 $OUT/gpu_suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python -u bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo BENCH_FAIL; tail -5 $OUT/bench_default.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench_default.json'));print('default', round(d['value']/1e6,2), 'M ops/s', round(d['ms_per_step'],1), 'ms', d['parity'], d['config'].get('lds_handover_docs'))"
for c in config3 config4 config5; do
  timeout -k 10 500 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-ingest > $OUT/${c}.json 2> $OUT/${c}.err || { echo FAIL $c; tail -5 $OUT/${c}.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/${c}.json'));print('$c', round(d['value']/1e6,2), 'M ops/s', round(d['ms_per_step'],1), 'ms', d['parity'])"
done
