#!/bin/bash
# SQ / TCC counter passes over the replay kernel (one counter group per run).
set -o pipefail
O=gpurun_out/sq
mkdir -p $O
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
B="bench.py --steps 1 --warmup 0 --no-cpu-baseline ${BENCH_ARGS:-}"
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_INST_CYCLES_SALU SQ_INSTS_SENDMSG SQ_BUSY_CYCLES" \
           "TCC_HIT_sum TCC_MISS_sum" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $O/p$i -o p$i -- python $B > $O/p$i.json 2> $O/p$i.err || { echo PMC${i}_FAIL; tail -5 $O/p$i.err; exit 1; }
done
python - <<'PY'
import csv, glob
for f in sorted(glob.glob("gpurun_out/sq/p*/p*_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if r["Kernel_Name"].startswith("mt_replay"):
            print(r["Counter_Name"], r["Counter_Value"])
PY
