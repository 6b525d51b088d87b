#!/bin/bash
# Round 4 A/B pass 3: the GPU suite with the lane-parallel packParent and the two-quad scour
# loads, the block-residency kernel without its in-wave HBM continuation (MT_BLK_NO_CONT=1:
# no scratch; config 3 hands no document over, config 2 hands over one, which that build
# leaves unfinished) vs the product on configs 2/3, and the zamboni breakdown (MT_PROFILE3).
set -o pipefail
OUT=gpurun_out/r04_ab3; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $OUT/gpu_suite.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -2 $OUT/gpu_suite.log; [ $rc -eq 0 ] || exit $rc
ab() {  # config variant lib
  MTGPU_LIB=$3 timeout -k 10 400 python -u bench.py --config $1 --steps 3 --warmup 1 --no-cpu-baseline --no-ingest > $OUT/${1}_$2.json 2> $OUT/${1}_$2.err || { echo FAIL $1 $2; tail -5 $OUT/${1}_$2.err; return 1; }
  python -c "import json;d=json.load(open('$OUT/${1}_$2.json'));print('$1 $2', round(d['value']/1e6,2), 'M ops/s', round(d['roofline']['kernel_ms'],1), 'ms', d['parity'])"
}
P=fluidframework_amd/libmtgpu.so
N=fluidframework_amd/libmtgpu_nocont.so
ab config3 product $P && ab config3 nocont $N && ab config3 product2 $P && ab config3 nocont2 $N || exit 1
ab config2 product $P && ab config2 nocont $N || exit 1
MT_PROF_FLAG=MT_PROFILE3 timeout -k 10 300 python -u tools/phase_profile.py config2 4096 3000 blk > $OUT/phase3_config2.txt 2>&1 || exit 1
cat $OUT/phase3_config2.txt
