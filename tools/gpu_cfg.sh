#!/bin/bash
# One bench config: bench line (with CPU baseline), kernel-trace stats, FETCH/WRITE PMC passes.
# usage: CFG=config3 bash tools/gpu_cfg.sh
set -o pipefail
CFG=${CFG:-config3}
O=gpurun_out/$CFG
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 500 python bench.py --config $CFG ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python bench.py --config $CFG --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > $O/kt_bench.json 2> $O/kt.err || { echo KT_FAIL; tail -5 $O/kt.err; exit 1; }
cat $O/kt/kt_kernel_stats.csv
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmcF -o pmcF -- python bench.py --config $CFG --steps 1 --warmup 0 --no-cpu-baseline ${BENCH_ARGS:-} > $O/pmcF.json 2> $O/pmcF.err || { echo PMCF_FAIL; tail -5 $O/pmcF.err; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmcW -o pmcW -- python bench.py --config $CFG --steps 1 --warmup 0 --no-cpu-baseline ${BENCH_ARGS:-} > $O/pmcW.json 2> $O/pmcW.err || { echo PMCW_FAIL; tail -5 $O/pmcW.err; exit 1; }
for f in F W; do (head -1 $O/pmc$f/pmc${f}_counter_collection.csv; grep "mt_" $O/pmc$f/pmc${f}_counter_collection.csv) > $O/pmc_$f.csv; done
echo done
