#!/bin/bash
# PMC counters for isolated conv launches (scripts/epi_bench.py shapes) — run on the GPU box:
#   scripts/pmc_conv.sh <outdir> "<shapes>" <cfg> [counters...]
set -e
ROOT=$(pwd)
OUT="$1"; SHAPES="$2"; CFG="$3"; shift 3
CTRS=${@:-"SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM"}
mkdir -p "$ROOT/$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --pmc $CTRS -d "$ROOT/$OUT" -o pmc --output-format csv -- \
  python3 "$ROOT/scripts/epi_bench.py" --shapes "$SHAPES" --cfg "$CFG" > "$ROOT/$OUT/log.txt" 2>&1
cd "$ROOT" && python3 scripts/pmc_summary.py "$OUT/pmc_counter_collection.csv" | grep -A12 "conv_fwd"
