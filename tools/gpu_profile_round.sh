#!/bin/bash
# Round measurement pass (one MI355X): for each bench config, the bench line,
# rocprofv3 --kernel-trace --stats of the same command, and the HBM traffic PMC
# passes (FETCH_SIZE and WRITE_SIZE in separate runs, MI355X_MICROARCH.md HBM
# section); SQ issue/wait counters for config 2.  Output: gpurun_out/<round>/.
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
  timeout -k 10 500 python $B > $O/${c}_bench.json 2> $O/${c}_bench.err || { echo BENCH_FAIL $c; tail -20 $O/${c}_bench.err; exit 1; }
  cat $O/${c}_bench.json
  timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${c}_kt -o kt -- python $B --steps 3 --warmup 1 --no-cpu-baseline > $O/${c}_kt_bench.json 2> $O/${c}_kt.err || { echo KT_FAIL $c; tail -5 $O/${c}_kt.err; exit 1; }
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/${c}_pmcF -o pmcF -- python $B --steps 1 --warmup 0 --no-cpu-baseline > $O/${c}_pmcF.json 2> $O/${c}_pmcF.err || { echo PMCF_FAIL $c; tail -5 $O/${c}_pmcF.err; exit 1; }
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/${c}_pmcW -o pmcW -- python $B --steps 1 --warmup 0 --no-cpu-baseline > $O/${c}_pmcW.json 2> $O/${c}_pmcW.err || { echo PMCW_FAIL $c; tail -5 $O/${c}_pmcW.err; exit 1; }
done
if [[ " $CFGS " == *" config2 "* ]]; then
  i=0
  for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES" \
             "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_INST_CYCLES_SALU SQ_BUSY_CYCLES" \
             "TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i+1))
    timeout -s KILL 200 rocprofv3 --pmc $grp --output-format csv -d $O/config2_sq$i -o sq$i -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/config2_sq$i.json 2> $O/config2_sq$i.err || { echo SQ${i}_FAIL; tail -5 $O/config2_sq$i.err; exit 1; }
  done
fi
find $O -name "*.csv" | sort
