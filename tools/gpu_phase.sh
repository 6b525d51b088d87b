#!/bin/bash
# Phase (s_memtime) profiles of the replay in both residencies.
set -o pipefail
O=gpurun_out/phase
mkdir -p $O
export PYTHONUNBUFFERED=1
for res in hbm lds; do
  for flag in MT_PROFILE MT_PROFILE2; do
    MT_PROF_FLAG=$flag timeout -k 10 300 python tools/phase_profile.py config2 ${DOCS:-1536} ${OPS:-3000} $res > $O/${flag}_$res.log 2>&1 || { echo FAIL $flag $res; tail -20 $O/${flag}_$res.log; exit 1; }
    cat $O/${flag}_$res.log
  done
done
