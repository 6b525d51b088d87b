#!/bin/bash
# north_star's target size on one GPU: config 5 with 1,048,576 Zipf documents (exact
# per-document pools from the generation's high-water marks), oracle digest parity on 4,096 of
# them, snapshot time reported; device memory before/after in the err log.
set -o pipefail
OUT=gpurun_out/${1:-north_star_1m}; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 1100 python -u bench.py --config config5 --docs 1048576 --steps 2 --warmup 1 --partition ${PARTITION:-8192:128} > $OUT/config5_1m.json 2> $OUT/config5_1m.err
rc=$?; echo "bench rc=$rc"; tail -c 1500 $OUT/config5_1m.json; tail -5 $OUT/config5_1m.err
exit $rc
