#!/bin/bash
# Round 4: the fixed engine (branch-free vis_rc; walks load leaf rows once, splits written from
# registers) on the whole GPU suite, then an A/B against the same tree with MT_LEAF_ONCE=0.
set -o pipefail
OUT=gpurun_out/r04_fix; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $OUT/gpu_suite.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -3 $OUT/gpu_suite.log
[ $rc -eq 0 ] || exit $rc
for c in config2 config3 config5; do
  for v in leaf0 product; do
    L=fluidframework_amd/libmtgpu.so; [ $v = leaf0 ] && L=fluidframework_amd/libmtgpu_leaf0.so
    MTGPU_LIB=$L timeout -k 10 400 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-ingest > $OUT/${c}_$v.json 2> $OUT/${c}_$v.err || { echo FAIL $c $v; tail -5 $OUT/${c}_$v.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/${c}_$v.json'));print('$c $v', round(d['value']/1e6,2), 'M ops/s', round(d['roofline']['kernel_ms'],1), 'ms', d['parity'], d.get('snapshot',{}).get('ms'))"
  done
done
