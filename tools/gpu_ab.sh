#!/bin/bash
# A/B bench of alternative engine builds against the default one, plus GPU parity.
# usage: tools/gpu_ab.sh [variant ...]   (variant = fluidframework_amd/libmtgpu_<variant>.so)
set -o pipefail
mkdir -p gpurun_out/ab
export PYTHONUNBUFFERED=1
O=gpurun_out/ab
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for v in default "$@"; do
  L=""; [ "$v" != default ] && L=$PWD/fluidframework_amd/libmtgpu_$v.so
  MTGPU_LIB=$L timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_$v.json 2> $O/bench_$v.err || { echo BENCH_${v}_FAIL; tail -20 $O/bench_$v.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_$v.json'));print('$v', round(d['value']/1e6,2),'Mops/s kernel', round(d['roofline']['kernel_ms'],1),'ms', d['parity'])"
done
if [ -f fluidframework_amd/libmtgpu_prof.so ]; then
  timeout -k 10 300 python tools/phase_profile.py config2 4096 > $O/phase.log 2>&1 || { echo PHASE_FAIL; tail -20 $O/phase.log; exit 1; }
  cat $O/phase.log
fi
