set -o pipefail
bash tools/gpu_ab_lib.sh r03s3_ab6nu fluidframework_amd/libmtgpu_nu.so config2 config3 && bash tools/gpu_ab_lib.sh r03s3_ab6o2 fluidframework_amd/libmtgpu_o2.so config2 config3
