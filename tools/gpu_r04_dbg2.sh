#!/bin/bash
# Round 4: the device-only INSERT_FAILED, second pass: the wide-load diagnostic build with
# 2 waves per SIMD (256 VGPRs: few spills) and with a full wait + fence before the leaf loads.
set -o pipefail
OUT=gpurun_out/r04_dbg2; mkdir -p $OUT
export PYTHONUNBUFFERED=1
fatal() { [ "$1" -eq 124 ] || [ "$1" -eq 137 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
for v in dbgw2 dbgfence; do
  MTGPU_LIB=fluidframework_amd/libmtgpu_$v.so timeout -k 10 300 python -u -m pytest -x -v --timeout 120 \
    --timeout-method thread -m gpu tests/test_client_api.py tests/test_gpu_parity.py > $OUT/$v.log 2>&1
  rc=$?; echo "$v rc=$rc"; grep -c WALKFAIL $OUT/$v.log; tail -3 $OUT/$v.log
  if fatal $rc; then exit $rc; fi
done
# where config 2's documents hand over from LDS blocks to HBM (product build)
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-ingest > $OUT/bench_c2.json 2> $OUT/bench_c2.err
rc=$?; echo "bench rc=$rc"; tail -c 600 $OUT/bench_c2.json
exit $rc
