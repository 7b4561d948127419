#!/bin/bash
# PMC counters of the ResNet-50 training step, one counter group per rocprofv3 pass (each pass is
# its own run: --pmc with --kernel-trace only). Run from the repo root on the GPU box:
#   scripts/pmc_step.sh <outdir> [bench args...]
# then: python3 scripts/pmc_report.py <outdir>
ROOT=$(pwd)
OUT="$ROOT/$1"; shift
mkdir -p "$OUT"
export PYTHONPATH=$ROOT
cd /tmp && export TMPDIR=/tmp
i=0
for ctrs in "SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
            "FETCH_SIZE" "WRITE_SIZE"; do
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $ctrs -d "$OUT/p$i" -o pmc --output-format csv -- \
    python3 "$ROOT/bench.py" --steps 2 --warmup 1 --graph 0 --plan 0 "$@" > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; exit 1; }
  i=$((i+1))
done
echo done
