# round-6 GPU call 14: the swizzled BN coefficient tables (bn.hip) and the stem input-halo weight
# gradient on the current tree: GPU test suite + smoke, bench A/B against a variant library with
# the previous bn.hip (DRN_KERNEL_LIB, 3 interleaved rounds), the data-parallel bench (DRN_BENCH_DP)
# with the round-5 stem choices (dbA) vs the re-tuned ones (shipped), and one SQ counter pass of
# each library for the BN applies' LDS bank conflicts.
set -o pipefail
ROOT=$(pwd)
O=$ROOT/gpurun_out/r6
mkdir -p $O
export PYTHONPATH=$ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/c14_tests.txt 2>&1 || { tail -30 $O/c14_tests.txt; exit 1; }
tail -3 $O/c14_tests.txt
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/c14_smoke.txt 2>&1 || { tail $O/c14_smoke.txt; exit 1; }
tail -2 $O/c14_smoke.txt
OLD=$ROOT/r6db/oldbn/libdrn_kernels.so
for i in 1 2 3; do
  timeout -k 10 200 python bench.py > $O/c14_x.json 2>> $O/c14.err || exit 1
  echo "new $(cut -c1-170 $O/c14_x.json)" >> $O/c14_ab.txt
  DRN_KERNEL_LIB=$OLD timeout -k 10 200 python bench.py > $O/c14_x.json 2>> $O/c14.err || exit 1
  echo "oldbn $(cut -c1-170 $O/c14_x.json)" >> $O/c14_ab.txt
done
for i in 1 2; do
  DRN_BENCH_DP=1 timeout -k 10 200 python bench.py > $O/c14_x.json 2>> $O/c14.err || exit 1
  echo "dp_halo $(cut -c1-170 $O/c14_x.json)" >> $O/c14_ab.txt
  DRN_BENCH_DP=1 DRN_TUNE_DB_SYSTEM=off DRN_TUNE_DB=$ROOT/r6db/dbA.json timeout -k 10 200 python bench.py > $O/c14_x.json 2>> $O/c14.err || exit 1
  echo "dp_r5stem $(cut -c1-170 $O/c14_x.json)" >> $O/c14_ab.txt
done
cat $O/c14_ab.txt
cd /tmp && export TMPDIR=/tmp
CT="SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $CT -d $O/c14_pmc_new -o pmc --output-format csv -- \
  python3 $ROOT/bench.py --steps 2 --warmup 1 --graph 0 --plan 0 > $O/c14_pmc_new.log 2>&1 || { echo "pmc new failed"; exit 1; }
DRN_KERNEL_LIB=$OLD timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $CT -d $O/c14_pmc_old -o pmc --output-format csv -- \
  python3 $ROOT/bench.py --steps 2 --warmup 1 --graph 0 --plan 0 > $O/c14_pmc_old.log 2>&1 || { echo "pmc old failed"; exit 1; }
echo pmc done
