#!/bin/bash
# Instruction-cache / issue counters of the default replay kernel (config 2, 3000 msgs/doc).
set -o pipefail
O=gpurun_out/ic2
mkdir -p $O
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
i=0
for grp in "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH" "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_IFETCH_LEVEL SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $O/p$i -o p$i -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline --ops 3000 > $O/p$i.json 2> $O/p$i.err || { echo PMC${i}_FAIL; tail -5 $O/p$i.err; exit 1; }
done
python - <<'PY'
import csv, glob
for f in sorted(glob.glob("gpurun_out/ic2/p*/p*_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if r["Kernel_Name"].startswith("mt_replay"):
            print(r["Kernel_Name"][:24], r["Counter_Name"], r["Counter_Value"])
PY
