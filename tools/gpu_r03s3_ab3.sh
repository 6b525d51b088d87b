set -o pipefail
PYTEST=1 bash tools/gpu_ab_lib.sh r03s3_ab3 fluidframework_amd/libmtgpu_v2.so config2 config3 || exit 1
mkdir -p gpurun_out/r03s3_prof
MT_PROF_FLAG=MT_PROFILE timeout -k 10 300 python -u tools/phase_profile.py config2 4096 3000 blk > gpurun_out/r03s3_prof/phase_c2.log 2>&1 || { tail -20 gpurun_out/r03s3_prof/phase_c2.log; exit 1; }
cat gpurun_out/r03s3_prof/phase_c2.log
MT_PROF_FLAG=MT_PROFILE3 timeout -k 10 300 python -u tools/phase_profile.py config2 4096 3000 blk > gpurun_out/r03s3_prof/phase3_c2.log 2>&1 || { tail -20 gpurun_out/r03s3_prof/phase3_c2.log; exit 1; }
cat gpurun_out/r03s3_prof/phase3_c2.log
