#!/bin/bash
# Per-op latency of long config-5-like documents (lag 32, 8 clients) by residency, plus config 5.
set -o pipefail
O=gpurun_out/${1:-longab}; mkdir -p $O
export PYTHONUNBUFFERED=1
for res in blk big hbm; do
  timeout -k 10 300 python -u bench.py --config config2 --docs 4 --ops 65536 --residency $res --steps 2 --warmup 1 --no-cpu-baseline --no-ingest > $O/long_$res.json 2> $O/long_$res.err || { tail -20 $O/long_$res.err; exit 1; }
  python -c "import json;d=json.load(open('$O/long_$res.json'));print('long $res', round(d['ms_per_step'],1), 'ms/step', round(d['ms_per_step']*1e3/65536,2), 'us/msg', d['parity'], d['config'].get('lds_handover_docs'))"
done
timeout -k 10 400 python -u bench.py --config config5 --steps 2 --warmup 1 --no-cpu-baseline > $O/config5.json 2> $O/config5.err || { tail -20 $O/config5.err; exit 1; }
python -c "import json;d=json.load(open('$O/config5.json'));print('config5', round(d['value']/1e6,2), 'M ops/s', round(d['ms_per_step'],1), 'ms', d['parity'], d['config']['msgs_max'])"
