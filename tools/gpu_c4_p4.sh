set -o pipefail
O=gpurun_out/r05_p4; mkdir -p $O
for f in 0 16; do
  MT_BIG_FLAGS=$f MT_PROF_FLAG=MT_PROFILE4 timeout -k 10 600 python tools/phase_config4.py 256 200000 5000 big > $O/p4_$f.txt 2>&1 || { tail $O/p4_$f.txt; exit 1; }
  echo "flags $f"; cat $O/p4_$f.txt
done
