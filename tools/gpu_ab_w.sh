#!/bin/bash
# Parity on the in-tree build, then time + WRITE_SIZE A/B against libmtgpu_base.so.
set -o pipefail
O=gpurun_out/abw
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
AB_LIBS=base bash tools/gpu_ab.sh || exit 1
AB_LIBS=base bash tools/gpu_ab.sh || exit 1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for v in base cur; do
  if [ $v = base ]; then export MTGPU_LIB=$PWD/fluidframework_amd/libmtgpu_base.so; else unset MTGPU_LIB; fi
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/${v}_w -o p -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/${v}_w.json 2> $O/${v}_w.err || { echo FAIL $v; tail -5 $O/${v}_w.err; exit 1; }
  python -c "
import csv
v=[float(r['Counter_Value']) for r in csv.DictReader(open('$O/${v}_w/p_counter_collection.csv')) if r['Kernel_Name'].startswith('mt_replay_blk_kernel') and r['Counter_Name']=='WRITE_SIZE']
print('$v WRITE_SIZE GB per launch', sum(v)/len(v)*1024/1e9)"
done
