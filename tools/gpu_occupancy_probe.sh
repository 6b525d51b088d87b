#!/bin/bash
# Per-message latency vs documents in flight (config 2 streams): is one wave's message
# bound by its own dependent chain or by sharing the SIMD with other waves?
set -o pipefail
OUT=gpurun_out/${1:-occ}; mkdir -p $OUT
for d in 4096 2048 1024 256 64; do
  timeout -k 10 300 python -u bench.py --docs $d --ops 3000 --steps 2 --warmup 1 --no-cpu-baseline --no-ingest > $OUT/c2_d$d.json 2> $OUT/c2_d$d.err || { tail -20 $OUT/c2_d$d.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/c2_d$d.json'));print('docs $d', round(d['value']/1e6,2), 'M ops/s', round(d['roofline']['kernel_ms'],2), 'ms', round(d['roofline']['kernel_ms']*1e3/3000,2), 'us/msg')"
done
