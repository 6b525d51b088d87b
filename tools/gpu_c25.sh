#!/bin/bash
# Config 2 and config 5 bench lines (no CPU baseline), after GPU parity.
set -o pipefail
O=gpurun_out/${1:-c25}; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for c in config2 config5; do
  timeout -k 10 400 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-ingest > $O/$c.json 2> $O/$c.err || { tail -20 $O/$c.err; exit 1; }
  python -c "import json;d=json.load(open('$O/$c.json'));print('$c', round(d['value']/1e6,3), 'M ops/s', round(d['ms_per_step'],1), 'ms', d['parity'])"
done
