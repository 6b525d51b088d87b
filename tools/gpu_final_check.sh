#!/bin/bash
# End-of-session check at the committed build: GPU parity, smoke, the default bench line
# (as the driver runs it) and the SQ instruction-mix / L2 counters of config 2.
set -o pipefail
O=gpurun_out/${1:-final}; mkdir -p $O
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail $O/bench_default.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_default.json'));print(round(d['value']/1e6,2), d['parity'], d['roofline']['traffic_source'])"
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_INST_CYCLES_SALU SQ_BUSY_CYCLES" \
           "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $grp --output-format csv -d $O/c2_sq$i -o sq$i -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-ingest > $O/c2_sq$i.json 2> $O/c2_sq$i.err || { echo SQ${i}_FAIL; tail -5 $O/c2_sq$i.err; exit 1; }
done
echo done
