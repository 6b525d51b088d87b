#!/bin/bash
# Where the replay kernel spends its issue slots: rocprofv3 host-trap PC sampling (beta) of a
# short config run, reduced per code-object offset by tools/pc_hot.py.  usage:
# tools/gpu_pc_sampling.sh <outdir under gpurun_out> <config> [ops]
set -o pipefail
O=gpurun_out/${1:-pcs}; C=${2:-config2}; OPS=${3:-3000}
mkdir -p $O
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -s KILL 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time \
  --pc-sampling-interval 1 --output-format csv -d $O/raw -o pcs -- python bench.py --config $C --ops $OPS --steps 1 \
  --warmup 0 --no-cpu-baseline --no-ingest > $O/bench.json 2> $O/bench.err
rc=$?; echo "pc sampling rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/bench.err; exit $rc; }
find $O/raw -name "*.csv" | head -5
