#!/bin/bash
# Round 3 A/B: product build (long-document scan in wave 0 for small windows, block cache
# compiled out) vs the cold-HBM-homes build (libmtgpu_v2.so) on configs 2 and 5; config 4;
# the fine-grained config-4 profile.
set -o pipefail
OUT=gpurun_out/r03_ab2; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_long_docs.py tests/test_gpu_parity.py tests/test_client_api.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for f in 0 4; do
  timeout -k 10 400 python -u bench.py --config config4 --steps 2 --warmup 1 --no-cpu-baseline --no-ingest --big-flags $f > $OUT/c4_f$f.json 2> $OUT/c4_f$f.err || { echo FAIL c4 $f; tail -20 $OUT/c4_f$f.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/c4_f$f.json'));print('config4 flags $f', round(d['value']/1e6,3), 'M ops/s', round(d['roofline']['kernel_ms'],1), 'ms', d['parity'])"
done
for v in prod v2; do
  L=""; [ $v = v2 ] && L=fluidframework_amd/libmtgpu_v2.so
  for c in config2 config5; do
    MTGPU_LIB=$L timeout -k 10 400 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-ingest > $OUT/${c}_$v.json 2> $OUT/${c}_$v.err || { echo FAIL $c $v; tail -20 $OUT/${c}_$v.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/${c}_$v.json'));print('$c $v', round(d['value']/1e6,3), 'M ops/s', round(d['roofline']['kernel_ms'],1), 'ms', d['parity'])"
  done
done
MT_PROF_FLAG=MT_PROFILE2 timeout -k 10 300 python -u tools/phase_config4.py 256 200000 5000 big > $OUT/c4_prof2.log 2>&1 || { tail -20 $OUT/c4_prof2.log; exit 1; }
cat $OUT/c4_prof2.log
