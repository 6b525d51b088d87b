#!/bin/bash
# Long documents (config-2 rules, 256 documents x 65,536 messages, the longest config-5 size) in the
# wide block-residency kernel (size class for every run) and in the block kernel with its in-wave
# continuation: microseconds per message and where documents leave LDS.
# usage: tools/gpu_long_probe.sh <outdir>
set -o pipefail
O=gpurun_out/${1:-longprobe}; mkdir -p $O
export PYTHONUNBUFFERED=1
for v in "wide --big-min-ops 1" "blk --big-min-ops 0 --cont-min 0"; do
  set -- $v; n=$1; shift
  timeout -k 10 400 python -u bench.py --config config2 --docs 256 --ops 65536 --steps 1 --warmup 0 --no-cpu-baseline --no-ingest "$@" > $O/$n.json 2> $O/$n.err || { echo FAIL $n; tail -20 $O/$n.err; exit 1; }
  python -c "import json;d=json.load(open('$O/$n.json'));r=d['roofline'];print('$n', round(r['kernel_ms'],1), 'ms', round(r['kernel_ms']*1e3/65536,2), 'us/msg', d['config']['lds_handover_docs'])"
done
