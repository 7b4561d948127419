# round-6 GPU call 8: split-K-capable 8-wave big tiles (gpu_variants/ks) vs the shipped configurations,
# full conv tuner on the stage-2..4 shapes, each library twice (interleaved)
set -o pipefail
mkdir -p gpurun_out/r6
for r in 1 2; do
  timeout -k 10 400 python -u scripts/ks_tile_probe.py --json gpurun_out/r6/ks_base_$r.json > gpurun_out/r6/ks_base_$r.txt 2>&1 && \
  DRN_KERNEL_LIB=$(pwd)/gpu_variants/ks/libdrn_kernels.so timeout -k 10 400 python -u scripts/ks_tile_probe.py --json gpurun_out/r6/ks_new_$r.json > gpurun_out/r6/ks_new_$r.txt 2>&1 || exit 1
done
