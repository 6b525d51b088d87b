#!/bin/bash
# Round 4: the GPU suite with the long-document parent cache (MT_G_BPC), config 4 A/B with the
# cache off at run time (--big-flags 8 = MT_BIGF_NO_BPC) vs on, and the MT_PROFILE4 computeU
# probes (window scan vs htBuild, parent-cache misses) on config 4's measured stream.
set -o pipefail
OUT=gpurun_out/r04_bpc; mkdir -p $OUT
export PYTHONUNBUFFERED=1
[ -n "$SKIP_SUITE" ] || timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $OUT/gpu_suite.log 2>&1
rc=$?; [ -n "$SKIP_SUITE" ] && rc=0; echo "suite rc=$rc"; tail -2 $OUT/gpu_suite.log; [ $rc -eq 0 ] || exit $rc
ab() {  # variant extra-args
  timeout -k 10 400 python -u bench.py --config config4 --steps 3 --warmup 1 --no-cpu-baseline --no-ingest $2 > $OUT/config4_$1.json 2> $OUT/config4_$1.err || { echo FAIL $1; tail -5 $OUT/config4_$1.err; return 1; }
  python -c "import json;d=json.load(open('$OUT/config4_$1.json'));print('config4 $1', round(d['value']/1e6,3), 'M ops/s', round(d['roofline']['kernel_ms'],1), 'ms', d['parity'])"
}
ab nobpc "--residency big --big-flags 8" && ab bpc "--residency big" && ab nobpc2 "--residency big --big-flags 8" && ab bpc2 "--residency big" || exit 1
MT_PROF_FLAG=MT_PROFILE4 timeout -k 10 300 python -u tools/phase_config4.py 256 200000 5000 big > $OUT/phase4_config4.txt 2>&1 || exit 1
cat $OUT/phase4_config4.txt
