#!/bin/bash
# Round-6 measurement pass (one MI355X): the full-scale manifest tests (configs 3-5), the default
# bench line as the driver runs it (config 2 with the ingest legs: Node JSON and Node parsed
# objects at full scale), then per config the rocprofv3 kernel-trace and PMC passes
# (tools/gpu_profile_r05.sh).  usage: tools/gpu_r06_measure.sh <outdir> [configs...]
set -o pipefail
R=${1:-r06_measure}; shift
O=gpurun_out/$R
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_full_scale_manifests.py \
    > $O/pytest_manifests.txt 2>&1 || { echo FAIL manifests; tail -30 $O/pytest_manifests.txt; exit 1; }
tail -3 $O/pytest_manifests.txt
timeout -k 10 900 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo FAIL bench; tail -20 $O/bench_default.err; exit 1; }
python -c "
import json; d=json.load(open('$O/bench_default.json'))
print('default', round(d['value']/1e6,2), 'M ops/s', round(d['ms_per_step'],2), 'ms', d['parity'][-50:])
ig = d.get('ingest', {})
for k in ('node_full_scale', 'node_objects_full_scale'):
    x = ig.get(k) or {}
    print(k, {q: x.get(q) for q in ('pack_msgs_per_s', 'e2e_msgs_per_s', 'digests_equal_bench', 'error')})"
[ $# -gt 0 ] && tools/gpu_profile_r05.sh $R/prof "$@"
exit 0
