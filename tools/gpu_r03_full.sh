#!/bin/bash
# Round 3 routine: the whole GPU suite and the smoke at this tree, then config 4 with the
# long-document switches (MT_BIGF_*), config 2, and config 5 with and without size classes.
set -o pipefail
OUT=gpurun_out/${1:-r03_full}; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
for f in ${C4FLAGS:-0 2 4 7}; do
  timeout -k 10 400 python -u bench.py --config config4 --steps 2 --warmup 1 --no-cpu-baseline --no-ingest --big-flags $f > $OUT/c4_f$f.json 2> $OUT/c4_f$f.err || { echo FAIL $f; tail -20 $OUT/c4_f$f.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/c4_f$f.json'));print('config4 big-flags $f', round(d['value']/1e6,3), 'M ops/s', round(d['roofline']['kernel_ms'],1), 'ms', d['parity'])"
done
timeout -k 10 400 python -u bench.py --config config2 --steps 5 --warmup 2 --no-cpu-baseline --no-ingest > $OUT/c2.json 2> $OUT/c2.err || { echo FAIL c2; tail -20 $OUT/c2.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/c2.json'));print('config2', round(d['value']/1e6,3), 'M ops/s', round(d['roofline']['kernel_ms'],1), 'ms', d['parity'])"
for b in ${C5BIG:-0 16384}; do
  timeout -k 10 400 python -u bench.py --config config5 --steps 2 --warmup 1 --no-cpu-baseline --no-ingest --big-min-ops $b > $OUT/c5_b$b.json 2> $OUT/c5_b$b.err || { echo FAIL c5 $b; tail -20 $OUT/c5_b$b.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/c5_b$b.json'));print('config5 big-min-ops $b', round(d['value']/1e6,3), 'M ops/s', round(d['roofline']['kernel_ms'],1), 'ms', d['parity'])"
done
