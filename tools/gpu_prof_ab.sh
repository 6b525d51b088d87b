#!/bin/bash
# Config-2 bench A/B (old vs current library) and the current library's phase profiles.
# usage: tools/gpu_prof_ab.sh <outdir> [old-lib]
set -o pipefail
O=gpurun_out/${1:-prof}; mkdir -p $O
export PYTHONUNBUFFERED=1
OLD=${2:-fluidframework_amd/libmtgpu_old.so}
CFGS=config2 ROUNDS=1 bash tools/gpu_lib_ab.sh ${1:-prof}/ab $OLD fluidframework_amd/libmtgpu.so || exit 1
timeout -k 10 300 python tools/phase_profile.py config2 4096 10000 blk > $O/new.txt 2>&1 || { tail $O/new.txt; exit 1; }
cat $O/new.txt
MT_PROF_FLAG=MT_PROFILE3 timeout -k 10 300 python tools/phase_profile.py config2 4096 10000 blk > $O/new3.txt 2>&1 || { tail $O/new3.txt; exit 1; }
cat $O/new3.txt
