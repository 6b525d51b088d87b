#!/bin/bash
# Round 4: where config 4's snapshot time goes (MT_SNAP_TIMING stage/emit split), then a PC
# sampling pass over config 2 (tools/gpu_pc_sampling.sh).
set -o pipefail
OUT=gpurun_out/r04_snap; mkdir -p $OUT
export PYTHONUNBUFFERED=1
MT_SNAP_TIMING=1 timeout -k 10 500 python -u bench.py --config config4 --steps 1 --warmup 0 --no-cpu-baseline --no-ingest > $OUT/config4.json 2> $OUT/config4.err || { echo FAIL; tail -5 $OUT/config4.err; exit 1; }
grep "mt_s" $OUT/config4.err | tail -8
python -c "import json;d=json.load(open('$OUT/config4.json'));print(d['snapshot'])"
bash tools/gpu_pc_sampling.sh pcs config2 3000
