#!/bin/bash
# Config 4 with and without the ancestor-chain guesses (MT_BIGF_NO_CHAIN = 16), GPU long-document
# parity tests first.  usage: tools/gpu_c4_chain_ab.sh <outdir>
set -o pipefail
O=gpurun_out/${1:-c4chain}; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_long_docs.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { tail -30 $O/pytest.log; exit $rc; }
for f in 0 16 0; do
  timeout -k 10 400 python -u bench.py --config config4 --steps 2 --warmup 1 --no-cpu-baseline --no-ingest --big-flags $f > $O/c4_$f.json 2> $O/c4_$f.err || { tail -20 $O/c4_$f.err; exit 1; }
  python -c "import json;d=json.load(open('$O/c4_$f.json'));print('config4 big-flags $f', round(d['value']/1e6,3), 'M ops/s', round(d['ms_per_step'],1), 'ms', d['parity'][-30:])"
done
