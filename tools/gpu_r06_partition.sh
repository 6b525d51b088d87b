#!/bin/bash
# Round 6: the automatic partition rule (mt_plan_partition) at bench's default for config 5 at
# 131,072 and 1,048,576 documents, the eight LPT shares of the 1,048,576-document N = 8 plan
# replayed in turn, and fixed specs beside them.  usage: tools/gpu_r06_partition.sh <outdir> [spec...]
set -o pipefail
OUT=gpurun_out/${1:-r06_part}; shift; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests \
    > $OUT/pytest_gpu.txt 2>&1 || { echo FAIL pytest; tail -30 $OUT/pytest_gpu.txt; exit 1; }
tail -2 $OUT/pytest_gpu.txt
summ() { python -c "import json;d=json.load(open('$1'));print('$2', round(d['value']/1e6,2), 'M ops/s', round(d['ms_per_step'],1), 'ms', d['config'].get('partition'), d['parity'][-48:])"; }
timeout -k 10 400 python -u bench.py --config config5 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/c5_auto.json 2> $OUT/c5_auto.err \
    || { echo FAIL c5; tail -20 $OUT/c5_auto.err; exit 1; }
summ $OUT/c5_auto.json "c5 131072 auto"
for t in "$@"; do
  n=${t/:/_}
  timeout -k 10 400 python -u bench.py --config config5 --steps 3 --warmup 1 --no-cpu-baseline --partition $t > $OUT/c5_$n.json 2> $OUT/c5_$n.err \
      || { echo FAIL $t; tail -20 $OUT/c5_$n.err; exit 1; }
  summ $OUT/c5_$n.json "c5 131072 $t"
done
timeout -k 10 420 python -u bench.py --config config5 --docs 1048576 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/c5_1m_auto.json 2> $OUT/c5_1m_auto.err \
    || { echo FAIL 1m; tail -20 $OUT/c5_1m_auto.err; exit 1; }
summ $OUT/c5_1m_auto.json "c5 1M auto"
timeout -k 10 600 python -u bench.py --config config5 --shares 8 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/c5_1m_shares8.json 2> $OUT/c5_1m_shares8.err \
    || { echo FAIL shares; tail -20 $OUT/c5_1m_shares8.err; exit 1; }
python -c "
import json;d=json.load(open('$OUT/c5_1m_shares8.json'))
for s in d['shares']: print('share', s['rank'], s['docs'], s['msgs'], round(s['ms_per_step'],1), 'ms', s['partition'])
print('projected node', round(d['value']/1e6,1), 'M ops/s, max step', round(d['ms_per_step'],1), 'ms;', d['parity'][-60:])"
