#!/bin/bash
# Config-5 digest parity vs the oracle's own generator at a reduced document count:
# the current tree, and (if present) the round-start tree in _old/.
set -o pipefail
O=gpurun_out/c5par; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python bench.py --config config5 --docs ${DOCS:-4096} --steps 1 --warmup 0 --cpu-seconds 2 --no-ingest > $O/new.json 2> $O/new.err || { tail $O/new.err; exit 1; }
python -c "import json;d=json.load(open('$O/new.json'));print('new', d['parity'])"
if [ -d _old ]; then
  (cd _old && timeout -k 10 300 python bench.py --config config5 --docs ${DOCS:-4096} --steps 1 --warmup 0 --cpu-seconds 2 --no-ingest > ../$O/old.json 2> ../$O/old.err) || { tail $O/old.err; exit 1; }
  python -c "import json;d=json.load(open('$O/old.json'));print('old', d['parity'])"
fi
