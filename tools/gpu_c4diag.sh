set -o pipefail
O=gpurun_out/c4diag; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
MT_PROF_FLAG=MT_PROFILE2 timeout -k 10 300 python tools/phase_config4.py 256 200000 5000 big > $O/p2.log 2>&1 || { tail $O/p2.log; exit 1; }
cat $O/p2.log
timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/tcc -o tcc -- python bench.py --config config4 --steps 1 --warmup 0 --no-cpu-baseline > $O/tcc.json 2> $O/tcc.err || { tail -5 $O/tcc.err; exit 1; }
echo done
