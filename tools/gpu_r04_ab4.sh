#!/bin/bash
# Round 4 pass 4: the GPU suite, then configs 2/3/5 with the batched text gather, the
# lane-parallel run lengths and the block-residency slack of 2*height + 10 (config 2's
# single hand-over document stays in LDS), and the zamboni breakdown (MT_PROFILE3).
set -o pipefail
OUT=gpurun_out/r04_ab4; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $OUT/gpu_suite.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -2 $OUT/gpu_suite.log; [ $rc -eq 0 ] || exit $rc
for c in config2 config3 config5; do
  timeout -k 10 400 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-ingest > $OUT/${c}.json 2> $OUT/${c}.err || { echo FAIL $c; tail -5 $OUT/${c}.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/${c}.json'));print('$c', round(d['value']/1e6,2), 'M ops/s', round(d['roofline']['kernel_ms'],1), 'ms', d['parity'], d['config'].get('lds_handover_docs'))"
done
MT_PROF_FLAG=MT_PROFILE3 timeout -k 10 300 python -u tools/phase_profile.py config2 4096 3000 blk > $OUT/phase3_config2.txt 2>&1 || exit 1
cat $OUT/phase3_config2.txt
