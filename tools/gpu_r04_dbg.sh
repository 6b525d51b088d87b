#!/bin/bash
# Round 4: the device-only INSERT_FAILED.  The wide-leaf-load diagnostic build (printf at the
# failing walk, fresh reloads beside the walk's values) on the test that failed in round 3,
# then the product build's GPU suite.
set -o pipefail
OUT=gpurun_out/r04_dbg; mkdir -p $OUT
export PYTHONUNBUFFERED=1
fatal() { [ "$1" -eq 124 ] || [ "$1" -eq 137 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
for v in dbgwide dbgfail; do
  MTGPU_LIB=fluidframework_amd/libmtgpu_$v.so timeout -k 10 300 python -u -m pytest -x -v --timeout 120 \
    --timeout-method thread -m gpu tests/test_client_api.py tests/test_gpu_parity.py > $OUT/$v.log 2>&1
  rc=$?; echo "$v rc=$rc"; grep -c WALKFAIL $OUT/$v.log; tail -3 $OUT/$v.log
  if fatal $rc; then exit $rc; fi
done
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $OUT/gpu_suite.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -3 $OUT/gpu_suite.log
exit $rc
