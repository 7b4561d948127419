#!/bin/bash
# PMC passes (one counter group per run) of the 14x14x256 3x3 layer: old LDS-DMA config vs halo.
OUT=${1:-gpurun_out/halopmc}
ROOT=$(pwd)
export PYTHONPATH=$ROOT
mkdir -p "$ROOT/$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for CT in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM" \
          "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"; do
  for cfg in 34 300; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $CT -d "$ROOT/$OUT/p$i" -o pmc --output-format csv -- \
      python3 "$ROOT/scripts/halo_pmc_run.py" 14 256 $cfg fwd 3 > "$ROOT/$OUT/p$i.log" 2>&1 || { tail -5 "$ROOT/$OUT/p$i.log"; exit 1; }
    python3 "$ROOT/scripts/pmc_summary.py" "$ROOT/$OUT/p$i/pmc_counter_collection.csv" | tee -a "$ROOT/$OUT/summary.txt"
  done
done
