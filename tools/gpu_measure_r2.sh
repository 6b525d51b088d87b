#!/bin/bash
# Round-2 measurement pass: phase profiles (config 2 and 4) and SQ/TCC counters (config 2).
set -o pipefail
O=gpurun_out/r2m
mkdir -p $O
export PYTHONUNBUFFERED=1
for flag in MT_PROFILE MT_PROFILE2 MT_PROFILE3; do
  MT_PROF_FLAG=$flag timeout -k 10 300 python tools/phase_profile.py config2 4096 3000 blk > $O/c2_${flag}.log 2>&1 || { echo FAIL $flag; tail -20 $O/c2_${flag}.log; exit 1; }
  cat $O/c2_${flag}.log
done
for flag in MT_PROFILE MT_PROFILE2; do
  MT_PROF_FLAG=$flag timeout -k 10 400 python tools/phase_config4.py 256 200000 5000 > $O/c4_${flag}.log 2>&1 || { echo FAIL c4 $flag; tail -20 $O/c4_${flag}.log; exit 1; }
  cat $O/c4_${flag}.log
done
