#!/bin/bash
# Round 3: stochastic PC sampling of the config-2 replay kernel (where the wave time goes,
# instruction by instruction, with stall reasons).
set -o pipefail
OUT=gpurun_out/r03_pcs; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
/opt/rocm/bin/rocprofv3 -L > $OUT/list.txt 2>&1 || true
grep -i -A12 "pc sampling\|pc_sampling" $OUT/list.txt | head -60
timeout -k 10 300 /opt/rocm/bin/rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles --pc-sampling-interval 262144 -d $OUT/raw -o pcs --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-ingest --docs 1024 > $OUT/run.log 2>&1 || { tail -30 $OUT/run.log; exit 1; }
tail -3 $OUT/run.log
find $OUT/raw -type f | head; du -sh $OUT/raw
