# round-6 GPU call 6: rebuild the kernel-selection database for the current kernel sources
set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 1150 bash scripts/gpu_make_db.sh gpurun_out/r6/db > gpurun_out/r6/db.txt 2>&1
