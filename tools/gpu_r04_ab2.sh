#!/bin/bash
# Round 4 A/B pass: the GPU suite at this tree, the no-newline flag (MT_NONL=0 vs product) on
# configs 2/3/5, the one-round-trip small-window scan (MT_G_ALLCH=0 vs product) on config 4, and
# per-phase cycle profiles (MT_PROFILE / MT_PROFILE2 builds) of configs 4 and 2.
set -o pipefail
OUT=gpurun_out/r04_ab2; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $OUT/gpu_suite.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -2 $OUT/gpu_suite.log; [ $rc -eq 0 ] || exit $rc
ab() {  # config variant lib
  MTGPU_LIB=$3 timeout -k 10 400 python -u bench.py --config $1 --steps 3 --warmup 1 --no-cpu-baseline --no-ingest > $OUT/${1}_$2.json 2> $OUT/${1}_$2.err || { echo FAIL $1 $2; tail -5 $OUT/${1}_$2.err; return 1; }
  python -c "import json;d=json.load(open('$OUT/${1}_$2.json'));print('$1 $2', round(d['value']/1e6,2), 'M ops/s', round(d['roofline']['kernel_ms'],1), 'ms', d['parity'])"
}
P=fluidframework_amd/libmtgpu.so
for c in config2 config3 config5; do ab $c nonl0 fluidframework_amd/libmtgpu_nonl0.so && ab $c product $P || exit 1; done
ab config4 allch0 fluidframework_amd/libmtgpu_allch0.so && ab config4 product $P || exit 1
MT_PROF_FLAG=MT_PROFILE timeout -k 10 300 python -u tools/phase_config4.py 256 200000 5000 big > $OUT/phase_config4.txt 2>&1 || exit 1
MT_PROF_FLAG=MT_PROFILE2 timeout -k 10 300 python -u tools/phase_config4.py 256 200000 5000 big > $OUT/phase2_config4.txt 2>&1 || exit 1
MT_PROF_FLAG=MT_PROFILE timeout -k 10 300 python -u tools/phase_profile.py config2 4096 3000 blk > $OUT/phase_config2.txt 2>&1 || exit 1
cat $OUT/phase_config4.txt $OUT/phase2_config4.txt $OUT/phase_config2.txt
