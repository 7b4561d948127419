#!/bin/bash
# PMC counters for one layer's conv kernels (run on the GPU box from the repo root):
#   scripts/pmc_layer.sh "<layer filter>" <outdir> [counters...]
set -e
ROOT=$(pwd)
FILTER="$1"; OUT="$2"; shift 2
CTRS=${@:-"SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"}
mkdir -p "$ROOT/$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --pmc $CTRS -d "$ROOT/$OUT" -o pmc --output-format csv -- \
  python3 "$ROOT/scripts/kernel_bench.py" --only "$FILTER" --iters 3 --no_bn > "$ROOT/$OUT/log.txt" 2>&1
