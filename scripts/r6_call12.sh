# round-6 GPU call 12: the packed stem's input-halo weight-gradient kernel: correctness (every
# pipeline vs the fp32 reference) and isolated time against the generic kernel
set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_ops_gpu.py -k "packed_stem or wgrad" > gpurun_out/r6/c12_tests.txt 2>&1 && \
timeout -k 10 300 python -u scripts/conv_bound_iso.py --run --case wgrad_stem --case wgrad_stem_halo3 --case wgrad_stem_halo4 --case wgrad_stem_halo3_768 > gpurun_out/r6/c12_stem_halo.txt 2>&1
