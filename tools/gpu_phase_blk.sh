#!/bin/bash
# Phase (s_memtime) profiles of the default block-residency replay (config 2 streams).
set -o pipefail
O=gpurun_out/phase_blk
mkdir -p $O
export PYTHONUNBUFFERED=1
for flag in MT_PROFILE MT_PROFILE2 MT_PROFILE3; do
  MT_PROF_FLAG=$flag timeout -k 10 300 python tools/phase_profile.py config2 ${DOCS:-4096} ${OPS:-3000} blk > $O/${flag}.log 2>&1 || { echo FAIL $flag; tail -20 $O/${flag}.log; exit 1; }
  cat $O/${flag}.log
done
