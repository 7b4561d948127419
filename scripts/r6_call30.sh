# round-6 GPU call 30: step profile of the current tree (fused stem, side-stream pool backward)
set -o pipefail
mkdir -p gpurun_out/r6
bash scripts/gpu_prof_step.sh gpurun_out/r6/c30
