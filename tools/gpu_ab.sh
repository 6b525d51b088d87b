#!/bin/bash
# A/B pass: GPU parity, config-2 and config-4 bench lines, config-4 phase profile.
set -o pipefail
O=gpurun_out/${1:-ab}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for c in config2 config4 ${EXTRA_CFGS}; do
  timeout -k 10 400 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-ingest > $O/$c.json 2> $O/$c.err || { tail -20 $O/$c.err; exit 1; }
  python -c "import json;d=json.load(open('$O/$c.json'));print('$c', round(d['value']/1e6,3), 'M ops/s', round(d['ms_per_step'],1), 'ms', d['parity'])"
done
if [ -f fluidframework_amd/libmtgpu_mt_profile.so ]; then
  MT_PROF_FLAG=MT_PROFILE timeout -k 10 400 python tools/phase_config4.py 256 200000 5000 big > $O/c4_phase.log 2>&1 || { tail -20 $O/c4_phase.log; exit 1; }
  cat $O/c4_phase.log
fi
