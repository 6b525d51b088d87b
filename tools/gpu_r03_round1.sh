#!/bin/bash
# Round-3 first measurement pass: GPU tests + default bench, configs 4/5, the residency probe
# for long documents and phase profiles (MT_PROFILE build) of one in blk and big residency.
set -o pipefail
bash tools/gpu_check.sh r03_c2 || exit 1
bash tools/gpu_bench_set.sh r03_ab1 config4 config5 || exit 1
bash tools/gpu_residency_probe.sh r03_res 30000 || exit 1
mkdir -p gpurun_out/r03_phase
for r in blk big; do
  timeout -k 10 300 python -u tools/phase_profile.py config2 512 30000 $r > gpurun_out/r03_phase/$r.log 2>&1 || { tail -20 gpurun_out/r03_phase/$r.log; exit 1; }
  cat gpurun_out/r03_phase/$r.log
done
