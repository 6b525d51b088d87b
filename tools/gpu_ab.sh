#!/bin/bash
# A/B of engine builds on one box: MTGPU_LIB=<alt .so> vs the in-tree libmtgpu.so.
set -o pipefail
mkdir -p gpurun_out/ab
for v in ${AB_LIBS:-base}; do
  MTGPU_LIB=$PWD/fluidframework_amd/libmtgpu_$v.so timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/ab/bench_$v.json 2> gpurun_out/ab/bench_$v.err || { echo BENCH_${v}_FAIL; tail -20 gpurun_out/ab/bench_$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab/bench_$v.json'));print('$v', round(d['value']/1e6,2),'Mops/s', round(d['roofline']['kernel_ms'],1),'ms')"
done
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/ab/bench_cur.json 2> gpurun_out/ab/bench_cur.err || { echo BENCH_FAIL; tail -20 gpurun_out/ab/bench_cur.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/ab/bench_cur.json'));print('cur', round(d['value']/1e6,2),'Mops/s', round(d['roofline']['kernel_ms'],1),'ms')"
