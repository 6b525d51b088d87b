#!/bin/bash
# Config-4 snapshot time, twice in separate processes, with the staging breakdown (MT_SNAP_TIMING).
# usage: tools/gpu_snap_timing.sh <outdir>
set -o pipefail
O=gpurun_out/${1:-snap}; mkdir -p $O
export PYTHONUNBUFFERED=1 MT_SNAP_TIMING=1
for i in 1 2; do
  timeout -k 10 400 python -u bench.py --config config4 --steps 1 --warmup 1 --no-cpu-baseline --no-ingest > $O/c4_$i.json 2> $O/c4_$i.err || { tail -20 $O/c4_$i.err; exit 1; }
  python -c "import json;d=json.load(open('$O/c4_$i.json'));print('config4 run $i', round(d['value']/1e6,2), 'M ops/s snapshot', d['snapshot'])"
  grep -E "mt_stage|mt_staged" $O/c4_$i.err | tail -12
done
