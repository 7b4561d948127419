#!/bin/bash
# Two PMC passes (plus a timing pass) over the conv kernels of selected layers, to compare the
# weight-gradient kernel's stall profile with the forward / data-gradient kernels of the same
# layer. Run from the repo root on the GPU box:
#   scripts/pmc_wgrad.sh <outdir> "<layer filter>" ["<layer filter>" ...]
ROOT=$(pwd)
OUT="$ROOT/$1"; shift
mkdir -p "$OUT"
export PYTHONPATH=$ROOT
cd /tmp && export TMPDIR=/tmp
i=0
for f in "$@"; do
  timeout -k 10 120 python3 "$ROOT/scripts/kernel_bench.py" --only "$f" --iters 20 --no_bn > "$OUT/time$i.txt" 2>&1 || { echo "timing $i failed"; exit 1; }
  j=0
  for ctrs in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU" \
              "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VMEM TCC_HIT_sum TCC_MISS_sum"; do
    timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $ctrs -d "$OUT/l${i}p$j" -o pmc --output-format csv -- \
      python3 "$ROOT/scripts/kernel_bench.py" --only "$f" --iters 2 --no_bn > "$OUT/l${i}p$j.log" 2>&1 || { echo "pass $i/$j failed"; tail -5 "$OUT/l${i}p$j.log"; exit 1; }
    python3 "$ROOT/scripts/pmc_summary.py" $(ls "$OUT"/l${i}p$j/*/*counter_collection.csv "$OUT"/l${i}p$j/*counter_collection.csv 2>/dev/null | head -1) > "$OUT/l${i}p$j.txt" || exit 1
    j=$((j+1))
  done
  i=$((i+1))
done
echo done
