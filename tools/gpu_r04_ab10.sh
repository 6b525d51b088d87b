#!/bin/bash
# Round 4 pass 10: the GPU suite, configs 2-5 at this tree (one-pass insert rows), then config 4
# with the multi-wave window scan from 128 entries (MT_G_MWMIN=128 build) against the product.
set -o pipefail
OUTDIR=r04_ab10 bash tools/gpu_r04_ab7.sh || exit 1
OUT=gpurun_out/r04_ab10
export PYTHONUNBUFFERED=1
MTGPU_LIB=fluidframework_amd/libmtgpu_mw128.so timeout -k 10 400 python -u bench.py --config config4 --steps 3 --warmup 1 --no-cpu-baseline --no-ingest > $OUT/config4_mw128.json 2> $OUT/config4_mw128.err || { echo FAIL mw128; tail -5 $OUT/config4_mw128.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/config4_mw128.json'));print('config4 mw128', round(d['value']/1e6,3), 'M ops/s', round(d['roofline']['kernel_ms'],1), 'ms', d['parity'])"
