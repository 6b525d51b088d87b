#!/bin/bash
# WRITE_SIZE / FETCH_SIZE of the replay kernel: an earlier engine build (MTGPU_LIB) vs the in-tree one.
set -o pipefail
O=gpurun_out/wab
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for v in old cur; do
  for k in WRITE_SIZE FETCH_SIZE; do
    if [ $v = old ]; then export MTGPU_LIB=$PWD/fluidframework_amd/libmtgpu_old.so; else unset MTGPU_LIB; fi
    timeout -s KILL 200 rocprofv3 --pmc $k --output-format csv -d $O/${v}_$k -o p -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/${v}_$k.json 2> $O/${v}_$k.err || { echo FAIL $v $k; tail -5 $O/${v}_$k.err; exit 1; }
    python -c "
import csv
v=[float(r['Counter_Value']) for r in csv.DictReader(open('$O/${v}_$k/p_counter_collection.csv')) if r['Kernel_Name'].startswith('mt_replay_blk_kernel') and r['Counter_Name']=='$k']
print('$v $k GB per launch', sum(v)/len(v)*1024/1e9, 'n', len(v))"
  done
done
