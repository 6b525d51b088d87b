#!/bin/bash
# Round-5 measurement pass (one MI355X): per config the bench line, rocprofv3 --kernel-trace
# --stats of the same command, FETCH_SIZE / WRITE_SIZE / SQ PMC passes (separate runs) reduced
# to <config>_traffic.json and <config>_sq_mix.txt.  Config 5's replay launch is the wide and the
# block kernels together (partitioned size classes): its traffic sums both, its SQ mix is the
# wide kernel's.  usage: tools/gpu_profile_r05.sh <round-dir> [configs...]
set -o pipefail
R=${1:-r05prof}; shift
CFGS=${@:-config2 config3 config4 config5}
O=gpurun_out/$R
mkdir -p $O
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for c in $CFGS; do
  B="bench.py --config $c"
  K=mt_replay_blk_kernel; KS=$K
  [ $c = config4 ] && K=mt_replay_big_kernel && KS=$K
  [ $c = config5 ] && K="mt_replay_blkw_kernel+mt_replay_blk_kernel" && KS=mt_replay_blkw_kernel
  X=""; [ $c = config2 ] && X="--no-ingest"
  timeout -k 10 600 python $B $X > $O/${c}_bench.json 2> $O/${c}_bench.err || { echo BENCH_FAIL $c; tail -20 $O/${c}_bench.err; exit 1; }
  python -c "import json;d=json.load(open('$O/${c}_bench.json'));print('$c', round(d['value']/1e6,2), 'M ops/s', round(d['ms_per_step'],1), 'ms', d['parity'][-40:])"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${c}_kt -o kt -- python $B --steps 3 --warmup 1 --no-cpu-baseline --no-ingest > $O/${c}_kt_bench.json 2> $O/${c}_kt.err || { echo KT_FAIL $c; tail -5 $O/${c}_kt.err; exit 1; }
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/${c}_pmcF -o pmcF -- python $B --steps 1 --warmup 0 --no-cpu-baseline --no-ingest > $O/${c}_pmcF.json 2> $O/${c}_pmcF.err || { echo PMCF_FAIL $c; tail -5 $O/${c}_pmcF.err; exit 1; }
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/${c}_pmcW -o pmcW -- python $B --steps 1 --warmup 0 --no-cpu-baseline --no-ingest > $O/${c}_pmcW.json 2> $O/${c}_pmcW.err || { echo PMCW_FAIL $c; tail -5 $O/${c}_pmcW.err; exit 1; }
  timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD --output-format csv -d $O/${c}_pmcS -o pmcS -- python $B --steps 1 --warmup 0 --no-cpu-baseline --no-ingest > $O/${c}_pmcS.json 2> $O/${c}_pmcS.err || { echo PMCS_FAIL $c; tail -5 $O/${c}_pmcS.err; exit 1; }
  python tools/sq_mix.py $(find $O/${c}_pmcS -name "*counter_collection.csv") $KS > $O/${c}_sq_mix.txt || echo SQMIX_FAIL $c
  D=$(python -c "import json;d=json.load(open('$O/${c}_pmcF.json'));print(d['config']['docs_per_gpu'], d['config'].get('msgs_per_doc', 0))")
  python tools/traffic_from_pmc.py $(find $O/${c}_pmcF -name "*counter_collection.csv") $(find $O/${c}_pmcW -name "*counter_collection.csv") $O/${c}_traffic.json $c $D "$K" || echo TRAFFIC_FAIL $c
done
find $O -name "*.csv" | sort
