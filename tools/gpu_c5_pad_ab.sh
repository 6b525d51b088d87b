set -o pipefail
O=gpurun_out/r05_pad; mkdir -p $O
export PYTHONUNBUFFERED=1
for spec in 256:224 2048:224 16384:224; do
  for lib in fluidframework_amd/libmtgpu.so fluidframework_amd/libmtgpu_pad.so; do
    n=$(basename $lib .so)_${spec/:/_}
    MTGPU_LIB=$lib timeout -k 10 300 python -u bench.py --config config5 --steps 2 --warmup 1 --no-cpu-baseline --no-ingest --partition $spec > $O/$n.json 2> $O/$n.err || { echo FAIL $n; tail -5 $O/$n.err; exit 1; }
    python -c "import json;d=json.load(open('$O/$n.json'));print('$n', round(d['value']/1e6,2), 'M ops/s', round(d['ms_per_step'],1), 'ms')"
  done
done
