#!/bin/bash
# Round 4 pass 6: the GPU suite with the bucketed parent table, then config 4 A/B: table with
# walk fill / table without walk fill (--big-flags 16) / no table (--big-flags 8).
set -o pipefail
OUT=gpurun_out/r04_ab6; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $OUT/gpu_suite.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -2 $OUT/gpu_suite.log; [ $rc -eq 0 ] || exit $rc
ab() {  # variant extra-args
  timeout -k 10 400 python -u bench.py --config config4 --steps 3 --warmup 1 --no-cpu-baseline --no-ingest --residency big $2 > $OUT/config4_$1.json 2> $OUT/config4_$1.err || { echo FAIL $1; tail -5 $OUT/config4_$1.err; return 1; }
  python -c "import json;d=json.load(open('$OUT/config4_$1.json'));print('config4 $1', round(d['value']/1e6,3), 'M ops/s', round(d['roofline']['kernel_ms'],1), 'ms', d['parity'])"
}
ab fill "" && ab nofill "--big-flags 16" && ab notable "--big-flags 8" && ab fill2 "" || exit 1
