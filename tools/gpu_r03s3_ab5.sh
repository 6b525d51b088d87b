set -o pipefail
PYTEST=1 bash tools/gpu_ab_lib.sh r03s3_ab5 fluidframework_amd/libmtgpu_v4.so config2 config3
