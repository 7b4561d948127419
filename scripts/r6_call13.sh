# round-6 GPU call 13: tune the packed stem's weight gradients with the input-halo pipelines
# (ns 9/10) into the re-keyed database, then A/B the bench: A = the round-5 choices (generic
# pipelines) carried over, B = the re-tuned entries. 3 interleaved rounds.
set -o pipefail
mkdir -p gpurun_out/r6
export PYTHONPATH=$(pwd)
cp distributed_resnet_tensorflow_amd/ops/tune_db.json gpurun_out/r6/dbB.json
DRN_TUNE_DB=$(pwd)/gpurun_out/r6/dbB.json timeout -k 10 600 python -u scripts/make_tune_db.py > gpurun_out/r6/c13_make.log 2>&1 || { tail gpurun_out/r6/c13_make.log; exit 1; }
cat gpurun_out/r6/c13_make.log
for i in 1 2 3; do
  DRN_TUNE_DB_SYSTEM=off DRN_TUNE_DB=$(pwd)/r6db/dbA.json timeout -k 10 200 python bench.py > gpurun_out/r6/c13_A.json 2>> gpurun_out/r6/c13.err || exit 1
  echo "A $(cut -c1-160 gpurun_out/r6/c13_A.json)" >> gpurun_out/r6/c13_ab.txt
  DRN_TUNE_DB_SYSTEM=off DRN_TUNE_DB=$(pwd)/gpurun_out/r6/dbB.json timeout -k 10 200 python bench.py > gpurun_out/r6/c13_B.json 2>> gpurun_out/r6/c13.err || exit 1
  echo "B $(cut -c1-160 gpurun_out/r6/c13_B.json)" >> gpurun_out/r6/c13_ab.txt
done
cat gpurun_out/r6/c13_ab.txt
