#!/bin/bash
# Round-6 A/B on one box: the round-5 library against this tree's (configs 2 and 4, alternating,
# no partition so both libraries run the same kernels), then the default bench line with both
# Node ingest legs.  usage: tools/gpu_r06_ab.sh <outdir>
set -o pipefail
O=gpurun_out/${1:-r06_ab}; mkdir -p $O
export PYTHONUNBUFFERED=1
for r in 1 2; do
  for lib in fluidframework_amd/libmtgpu_r05.so fluidframework_amd/libmtgpu.so; do
    for c in config2 config4; do
      n=$(basename $lib .so)_${c}_$r
      MTGPU_LIB=$lib timeout -k 10 300 python -u bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline --no-ingest --partition off > $O/$n.json 2> $O/$n.err || { echo FAIL $n; tail -20 $O/$n.err; exit 1; }
      python -c "import json;d=json.load(open('$O/$n.json'));print('$n', round(d['value']/1e6,2), 'M ops/s', round(d['ms_per_step'],1), 'ms', d['parity'][-24:])"
    done
  done
done
timeout -k 10 900 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo FAIL bench; tail -20 $O/bench_default.err; exit 1; }
python -c "
import json; d=json.load(open('$O/bench_default.json'))
print('default', round(d['value']/1e6,2), 'M ops/s', round(d['ms_per_step'],2), 'ms', d['parity'][-50:])
ig = d.get('ingest', {})
for k in ('node_full_scale', 'node_objects_full_scale'):
    x = ig.get(k) or {}
    print(k, {q: x.get(q) for q in ('pack_msgs_per_s', 'e2e_msgs_per_s', 'digests_equal_bench', 'error')})"
