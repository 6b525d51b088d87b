#!/bin/bash
# Config 2 / 5 bench A/B of two engine libraries plus a WRITE_SIZE pass of each on config 2.
# usage: tools/gpu_write_ab.sh <outdir> <libA> <libB>
set -o pipefail
O=gpurun_out/${1:-wab}; A=$2; B=$3; mkdir -p $O
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
CFGS="config2 config5" ROUNDS=1 bash tools/gpu_lib_ab.sh ${1:-wab}/ab $A $B || exit 1
for lib in $A $B; do
  n=$(basename $lib .so)
  MTGPU_LIB=$lib timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/${n}_pmcW -o pmcW -- python bench.py --config config2 --steps 1 --warmup 0 --no-cpu-baseline --no-ingest > $O/${n}_pmcW.json 2> $O/${n}_pmcW.err || { echo PMCW_FAIL $n; tail -5 $O/${n}_pmcW.err; exit 1; }
  python -c "
import csv,sys
sys.path.insert(0,'tools')
from traffic_from_pmc import bare
import glob
f=glob.glob('$O/${n}_pmcW/**/*counter_collection.csv', recursive=True)[0]
v=[float(r['Counter_Value']) for r in csv.DictReader(open(f)) if bare(r['Kernel_Name'])=='mt_replay_blk_kernel' and r['Counter_Name']=='WRITE_SIZE']
print('$n config2 WRITE_SIZE GB per launch', round(sum(v)/len(v)*1024/1e9, 2))
"
done
