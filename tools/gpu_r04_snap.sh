#!/bin/bash
# Round 4: where config 4's snapshot time goes (MT_SNAP_TIMING stage/emit split)
set -o pipefail
OUT=gpurun_out/r04_snap; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $OUT/gpu_suite.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -2 $OUT/gpu_suite.log; [ $rc -eq 0 ] || exit $rc
MT_SNAP_TIMING=1 timeout -k 10 500 python -u bench.py --config config4 --steps 1 --warmup 0 --no-cpu-baseline --no-ingest > $OUT/config4.json 2> $OUT/config4.err || { echo FAIL; tail -5 $OUT/config4.err; exit 1; }
grep "mt_s" $OUT/config4.err | tail -30
python -c "import json;d=json.load(open('$OUT/config4.json'));print(d['snapshot'])"
