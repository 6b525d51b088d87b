#!/bin/bash
# Long-document residency check: GPU parity, config-4 bench (big vs blk), config-4 phase
# profile in big mode, config-2 SQ instruction-mix counters.
set -o pipefail
O=gpurun_out/${1:-big}
mkdir -p $O
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 400 python -u bench.py --config config4 --steps 2 --warmup 1 --no-cpu-baseline > $O/c4_big.json 2> $O/c4_big.err || { tail -20 $O/c4_big.err; exit 1; }
python -c "import json;d=json.load(open('$O/c4_big.json'));print('config4 big', round(d['value']/1e6,3), 'M ops/s', d['ms_per_step'], d['parity'])"
MT_PROF_FLAG=MT_PROFILE timeout -k 10 400 python tools/phase_config4.py 256 200000 5000 big > $O/c4_phase_big.log 2>&1 || { tail -20 $O/c4_phase_big.log; exit 1; }
cat $O/c4_phase_big.log
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_INST_CYCLES_SALU SQ_BUSY_CYCLES" \
           "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $grp --output-format csv -d $O/c2_sq$i -o sq$i -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-ingest > $O/c2_sq$i.json 2> $O/c2_sq$i.err || { echo SQ${i}_FAIL; tail -5 $O/c2_sq$i.err; exit 1; }
done
find $O -name "*counter_collection.csv" | sort
