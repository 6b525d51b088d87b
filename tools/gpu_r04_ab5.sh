#!/bin/bash
# Round 4 pass 5: the GPU suite with the open-addressing parent table (walk-populated), then
# config 4 A/B: table on / off (--big-flags 8) and the multi-wave window scan from 128 / 256
# entries (MT_G_MWMIN builds) instead of 512.
set -o pipefail
OUT=gpurun_out/r04_ab5; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $OUT/gpu_suite.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -2 $OUT/gpu_suite.log; [ $rc -eq 0 ] || exit $rc
ab() {  # variant lib extra-args
  MTGPU_LIB=$2 timeout -k 10 400 python -u bench.py --config config4 --steps 3 --warmup 1 --no-cpu-baseline --no-ingest --residency big $3 > $OUT/config4_$1.json 2> $OUT/config4_$1.err || { echo FAIL $1; tail -5 $OUT/config4_$1.err; return 1; }
  python -c "import json;d=json.load(open('$OUT/config4_$1.json'));print('config4 $1', round(d['value']/1e6,3), 'M ops/s', round(d['roofline']['kernel_ms'],1), 'ms', d['parity'])"
}
P=fluidframework_amd/libmtgpu.so
ab table $P "" && ab notable $P "--big-flags 8" && ab mw128 fluidframework_amd/libmtgpu_mw128.so "" && ab mw256 fluidframework_amd/libmtgpu_mw256.so "" && ab table2 $P "" || exit 1
