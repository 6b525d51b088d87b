#!/bin/bash
# Debug: where the GPU and the host emulation first disagree on a cfg2 stream (bisection
# builds loaded through MTGPU_LIB).
set -o pipefail
OUT=gpurun_out/dbg2; mkdir -p $OUT
export PYTHONUNBUFFERED=1
for v in a b; do
  lib=fluidframework_amd/libmtgpu_bisect_$v.so
  echo "== $lib"
  MTGPU_LIB=$lib DBG_NDOC=4 DBG_SEED=41 DBG_PREFIX=1 timeout -k 10 300 python -u tools/dbg_first_divergence.py cfg2 1500 > $OUT/prefix_$v.log 2>&1; tail -12 $OUT/prefix_$v.log
done
