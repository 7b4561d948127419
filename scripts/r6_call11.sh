# round-6 GPU call 11: bound isolation of the packed stem (forward and weight gradient)
set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 600 python -u scripts/conv_bound_iso.py --all --case fwd_stem --case wgrad_stem --case wgrad3x3_28 --out gpurun_out/r6/conv_bound_iso_stem.txt > gpurun_out/r6/conv_bound_iso_stem.log 2>&1
