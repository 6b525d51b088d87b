#!/bin/bash
# Instruction-cache and issue counters of the replay kernels (both residencies).
set -o pipefail
O=gpurun_out/ic
mkdir -p $O
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1 || echo "LIST rc=$?"
grep -o -E "\b(SQC?_[A-Z_0-9]+)\b" $O/counters.txt | sort -u > $O/names.txt || true
grep -E "ICACHE|IFETCH|INST_LEVEL|WAIT_INST|LDS|SQC_TC" $O/names.txt | tr '\n' ' '; echo
IC=""
for c in SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_IFETCH_LEVEL SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES; do grep -qx $c $O/names.txt && IC="$IC $c"; done
echo "pass:$IC"
for res in hbm lds; do
  timeout -s KILL 120 rocprofv3 --pmc $IC --output-format csv -d $O/$res -o p -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline --ops 3000 --residency $res > $O/$res.json 2> $O/$res.err || { echo PMC_FAIL; tail -5 $O/$res.err; exit 1; }
  python - <<PY
import csv
for r in csv.DictReader(open("$O/$res/p_counter_collection.csv")):
    if "replay" in r["Kernel_Name"]:
        print("$res", r["Kernel_Name"][:22], r["Counter_Name"], r["Counter_Value"])
PY
done
