#!/bin/bash
# Partitioned size classes (mt_set_partition): the parity tests, then config 5 with the long
# documents on reserved CUs, one per SIMD, at several (min messages : CUs) splits.
# usage: tools/gpu_partition_ab.sh <outdir under gpurun_out> [splits...]
set -o pipefail
OUT=gpurun_out/${1:-partition}; shift
SPLITS=${@:-off 48000:64 35000:128 28000:192}
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_long_docs.py -k "size_classes or partition" > $OUT/pytest.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for p in $SPLITS; do
  n=${p/:/_}
  timeout -k 10 400 python -u bench.py --config config5 --steps 3 --warmup 1 --no-cpu-baseline --no-ingest --partition $p > $OUT/config5_$n.json 2> $OUT/config5_$n.err || { echo FAIL $p; tail -5 $OUT/config5_$n.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/config5_$n.json'));print('config5 $p', round(d['value']/1e6,2), 'M ops/s', round(d['ms_per_step'],1), 'ms', d['parity'])"
done
