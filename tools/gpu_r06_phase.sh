#!/bin/bash
# Per-phase shader-clock cycles per message of the block-residency kernel (MT_PROFILE and
# MT_PROFILE3 diagnostic builds, prebuilt in-tree), config 2 at full size and config 5's
# long-document shape.  usage: tools/gpu_r06_phase.sh <outdir>
set -o pipefail
O=gpurun_out/${1:-r06_phase}; mkdir -p $O
export PYTHONUNBUFFERED=1
for f in MT_PROFILE MT_PROFILE3; do
  MT_PROF_FLAG=$f timeout -k 10 300 python tools/phase_profile.py config2 4096 10000 blk > $O/config2_$f.txt 2> $O/config2_$f.err || { echo FAIL $f; tail -20 $O/config2_$f.err; exit 1; }
  cat $O/config2_$f.txt
done
