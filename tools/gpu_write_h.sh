#!/bin/bash
# WRITE_SIZE of the replay kernel and a bench line for an alternate build (MTGPU_LIB).
set -o pipefail
O=gpurun_out/wh
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
export MTGPU_LIB=$PWD/fluidframework_amd/libmtgpu_h126.so
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w -o p -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/w.json 2> $O/w.err || { echo FAIL; tail -5 $O/w.err; exit 1; }
python -c "
import csv
v=[float(r['Counter_Value']) for r in csv.DictReader(open('$O/w/p_counter_collection.csv')) if r['Kernel_Name'].startswith('mt_replay_blk_kernel') and r['Counter_Name']=='WRITE_SIZE']
print('h126 WRITE_SIZE GB per launch', sum(v)/len(v)*1024/1e9)"
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/b.json 2> $O/b.err || { echo BENCH_FAIL; tail -5 $O/b.err; exit 1; }
python -c "import json;d=json.load(open('$O/b.json'));print('h126', round(d['value']/1e6,2),'Mops/s', d['config'].get('lds_handover_docs'))"
