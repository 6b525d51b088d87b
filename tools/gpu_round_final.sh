#!/bin/bash
# GPU parity, then the round's profile pass for the given configs (tools/gpu_profile_round.sh).
# usage: tools/gpu_round_final.sh <round> configs...
set -o pipefail
R=$1; shift
mkdir -p gpurun_out/$R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$R/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/$R/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/$R/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$R/smoke.log 2>&1 || { cat gpurun_out/$R/smoke.log; exit 1; }
cat gpurun_out/$R/smoke.log
bash tools/gpu_profile_round.sh $R "$@"
