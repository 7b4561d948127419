#!/bin/bash
# Step A/B: one weight-gradient workgroup per CU (LDS floor) vs the default.
OUT=${1:-gpurun_out/ab5}
export PYTHONPATH=$(pwd)
mkdir -p "$OUT"
bash scripts/gpu_env_ab.sh "$OUT" ${ROUNDS:-3} "def=DRN_WGRAD_LDS_MIN=0" "lds82k=DRN_WGRAD_LDS_MIN=83968" || exit 1
