#!/bin/bash
# Per-message cost of long documents by residency: the same stream (config-2 rules, 512
# documents x N messages) under blk (hands over to HBM), big and hbm residency.
# usage: tools/gpu_residency_probe.sh <outdir-under-gpurun_out> [msgs]
set -o pipefail
OUT=gpurun_out/${1:-resprobe}; N=${2:-30000}
mkdir -p $OUT
export PYTHONUNBUFFERED=1
for r in blk big hbm; do
  timeout -k 10 300 python -u bench.py --config config2 --docs 512 --ops $N --residency $r --steps 1 --warmup 0 --no-cpu-baseline --no-ingest > $OUT/$r.json 2> $OUT/$r.err || { echo FAIL $r; tail -20 $OUT/$r.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/$r.json'));print('$r', round(d['value']/1e6,3), 'M ops/s', round(d['roofline']['kernel_ms'],1), 'ms', round(d['roofline']['kernel_ms']*1e3/$N,2), 'us/msg', d['parity'])"
done
