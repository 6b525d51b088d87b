#!/bin/bash
# End-of-round measurement: configs 2 and 3 (bench with CPU baseline, kernel-trace
# stats, FETCH_SIZE / WRITE_SIZE PMC passes), then configs 4 and 5 bench lines.
set -o pipefail
CFG=config2 bash tools/gpu_cfg.sh || exit 1
CFG=config3 bash tools/gpu_cfg.sh || exit 1
for c in config4 config5; do
  mkdir -p gpurun_out/$c
  timeout -k 10 500 python bench.py --config $c > gpurun_out/$c/bench.json 2> gpurun_out/$c/bench.err || { echo BENCH_${c}_FAIL; tail -20 gpurun_out/$c/bench.err; exit 1; }
  cat gpurun_out/$c/bench.json
done
