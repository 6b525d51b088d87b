#!/bin/bash
# Library A/B with write/fetch accounting on one box: per library the config's bench line
# (partition off, alternating rounds), then a FETCH_SIZE and a WRITE_SIZE pass (separate
# rocprofv3 runs) reduced to <lib>_<config>_traffic.json.
# usage: CFGS="config2" ROUNDS=2 tools/gpu_r06_pmcab.sh <outdir> <lib.so>...
set -o pipefail
O=gpurun_out/${1:-r06_pmcab}; shift; mkdir -p $O
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
CFGS=${CFGS:-config2} tools/gpu_r06_libs.sh $(basename $O) "$@" || exit 1
for lib in "$@"; do
  for c in ${CFGS:-config2}; do
    n=$(basename $lib .so)_${c}
    K=mt_replay_blk_kernel; [ $c = config4 ] && K=mt_replay_big_kernel
    B="bench.py --config $c --steps 1 --warmup 0 --no-cpu-baseline --no-ingest --partition off"
    MTGPU_LIB=$lib timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/${n}_pmcF -o pmcF -- python $B > $O/${n}_pmcF.json 2> $O/${n}_pmcF.err || { echo PMCF_FAIL $n; tail -5 $O/${n}_pmcF.err; exit 1; }
    MTGPU_LIB=$lib timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/${n}_pmcW -o pmcW -- python $B > $O/${n}_pmcW.json 2> $O/${n}_pmcW.err || { echo PMCW_FAIL $n; tail -5 $O/${n}_pmcW.err; exit 1; }
    D=$(python -c "import json;d=json.load(open('$O/${n}_pmcF.json'));print(d['config']['docs_per_gpu'], d['config'].get('msgs_per_doc', 0))")
    python tools/traffic_from_pmc.py $(find $O/${n}_pmcF -name "*counter_collection.csv") $(find $O/${n}_pmcW -name "*counter_collection.csv") $O/${n}_traffic.json $c $D "$K" || echo TRAFFIC_FAIL $n
    python -c "import json;t=json.load(open('$O/${n}_traffic.json'));print('$n', 'fetch', round(t['fetch_bytes_raw']/1e9,2), 'write', round(t['write_bytes']/1e9,2), 'traffic', round(t['traffic_bytes']/1e9,2), 'GB')"
  done
done
