#!/bin/bash
# Diagnose the replay kernel: occupancy sweep, SQ/SQC/TCC counters, kernel-trace stats.
set -o pipefail
mkdir -p gpurun_out/r5
export PYTHONUNBUFFERED=1
O=gpurun_out/r5
B="bench.py --steps 1 --warmup 0 --no-cpu-baseline --ops 2000"
for d in 1024 2048 4096 8192; do
  timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --ops 3000 --docs $d > $O/sweep_$d.json 2> $O/sweep_$d.err || { echo SWEEP_FAIL $d; tail $O/sweep_$d.err; exit 1; }
  python -c "import json;d=json.load(open('$O/sweep_$d.json'));print($d, round(d['value']/1e6,2),'Mops/s', round(d['roofline']['kernel_ms'],1),'ms')"
done
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1 || echo "LIST rc=$?"
grep -o -E "\b(SQC?_[A-Z_0-9]+|TCC_[A-Z_0-9]+|TCP_[A-Z_0-9]+)\b" $O/counters.txt | sort -u > $O/counter_names.txt || true
wc -l $O/counter_names.txt
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES --output-format csv -d $O/pmcA -o pmcA -- python $B > $O/pmcA.log 2>&1 || { echo PMCA_FAIL; tail -5 $O/pmcA.log; exit 1; }
IC=""
for c in SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_DCACHE_HITS SQC_DCACHE_MISSES; do grep -qx $c $O/counter_names.txt && IC="$IC $c"; done
echo "SQC pass:$IC"
if [ -n "$IC" ]; then
  timeout -s KILL 120 rocprofv3 --pmc $IC --output-format csv -d $O/pmcB -o pmcB -- python $B > $O/pmcB.log 2>&1 || { echo PMCB_FAIL; tail -5 $O/pmcB.log; exit 1; }
fi
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmcC -o pmcC -- python $B > $O/pmcC.log 2>&1 || { echo PMCC_FAIL; tail -5 $O/pmcC.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmcD -o pmcD -- python $B > $O/pmcD.log 2>&1 || { echo PMCD_FAIL; tail -5 $O/pmcD.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/kt_bench.json 2> $O/kt.err || { echo KT_FAIL; tail -5 $O/kt.err; exit 1; }
tail -1 $O/kt_bench.json
find $O -name "*.csv" | head -20
