#!/bin/bash
# Round measurement pass (one MI355X): for each bench config, the bench line (with the
# CPU baseline), rocprofv3 --kernel-trace --stats of the same command, and the HBM
# traffic PMC passes (FETCH_SIZE and WRITE_SIZE in separate runs, MI355X_MICROARCH.md HBM
# section), reduced to <config>_traffic.json, and an SQ pass (wave cycles parked / stalled /
# issuing, instruction mix) reduced to <config>_sq_mix.txt.  Output: gpurun_out/<round>/.
# usage: tools/gpu_profile_round.sh r02 [configs...]
set -o pipefail
R=${1:-r02}; shift
CFGS=${@:-config2 config3 config4 config5}
O=gpurun_out/$R
mkdir -p $O
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for c in $CFGS; do
  B="bench.py --config $c"
  K=mt_replay_blk_kernel; [ $c = config4 ] && K=mt_replay_big_kernel
  timeout -k 10 500 python $B > $O/${c}_bench.json 2> $O/${c}_bench.err || { echo BENCH_FAIL $c; tail -20 $O/${c}_bench.err; exit 1; }
  cat $O/${c}_bench.json
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${c}_kt -o kt -- python $B --steps 3 --warmup 1 --no-cpu-baseline --no-ingest > $O/${c}_kt_bench.json 2> $O/${c}_kt.err || { echo KT_FAIL $c; tail -5 $O/${c}_kt.err; exit 1; }
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/${c}_pmcF -o pmcF -- python $B --steps 1 --warmup 0 --no-cpu-baseline --no-ingest > $O/${c}_pmcF.json 2> $O/${c}_pmcF.err || { echo PMCF_FAIL $c; tail -5 $O/${c}_pmcF.err; exit 1; }
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/${c}_pmcW -o pmcW -- python $B --steps 1 --warmup 0 --no-cpu-baseline --no-ingest > $O/${c}_pmcW.json 2> $O/${c}_pmcW.err || { echo PMCW_FAIL $c; tail -5 $O/${c}_pmcW.err; exit 1; }
  timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD --output-format csv -d $O/${c}_pmcS -o pmcS -- python $B --steps 1 --warmup 0 --no-cpu-baseline --no-ingest > $O/${c}_pmcS.json 2> $O/${c}_pmcS.err || { echo PMCS_FAIL $c; tail -5 $O/${c}_pmcS.err; exit 1; }
  python tools/sq_mix.py $(find $O/${c}_pmcS -name "*counter_collection.csv") $K > $O/${c}_sq_mix.txt || echo SQMIX_FAIL $c
  D=$(python -c "import json;d=json.load(open('$O/${c}_pmcF.json'));print(d['config']['docs_per_gpu'], d['config'].get('msgs_per_doc', 0))")
  python tools/traffic_from_pmc.py $(find $O/${c}_pmcF -name "*counter_collection.csv") $(find $O/${c}_pmcW -name "*counter_collection.csv") $O/${c}_traffic.json $c $D $K || echo TRAFFIC_FAIL $c
done
find $O -name "*.csv" | sort
