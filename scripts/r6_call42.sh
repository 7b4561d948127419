# round-6 GPU call 42: final-tree PMC passes of the ResNet-50 step (scripts/pmc_step.sh: one counter
# group per rocprofv3 run, --pmc with --kernel-trace only), per-dispatch roofline + family summary
set -o pipefail
ROOT=$(pwd)
O=gpurun_out/r6/c42_pmc
mkdir -p gpurun_out/r6
bash scripts/pmc_step.sh $O > gpurun_out/r6/c42_pmc.log 2>&1 || { tail -20 gpurun_out/r6/c42_pmc.log; exit 1; }
python3 scripts/pmc_dispatch.py $O > gpurun_out/r6/c42_pmc_dispatch.txt 2>&1 || { tail gpurun_out/r6/c42_pmc_dispatch.txt; exit 1; }
python3 scripts/pmc_report.py $O > gpurun_out/r6/c42_pmc_by_family.txt 2>&1 || true
head -12 gpurun_out/r6/c42_pmc_dispatch.txt
