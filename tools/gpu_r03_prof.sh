#!/bin/bash
# Round 3: phase (MT_PROFILE) and fine-grained (MT_PROFILE2) profiles of config 4's measured
# stream in big residency; the diagnostic libraries are built on the CPU beforehand.
set -o pipefail
OUT=gpurun_out/r03_prof; mkdir -p $OUT
export PYTHONUNBUFFERED=1
for f in MT_PROFILE MT_PROFILE2; do
  MT_PROF_FLAG=$f timeout -k 10 300 python -u tools/phase_config4.py 256 200000 5000 big > $OUT/c4_$f.log 2>&1 || { tail -20 $OUT/c4_$f.log; exit 1; }
  cat $OUT/c4_$f.log
done
