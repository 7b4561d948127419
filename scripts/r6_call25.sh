# round-6 GPU call 25: fused stem iteration: correctness + isolated time (+ SQ counters)
set -o pipefail
ROOT=$(pwd)
O=$ROOT/gpurun_out/r6
mkdir -p $O
export PYTHONPATH=$ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_ops_gpu.py \
  -k "fused_stem" > $O/c25_tests.txt 2>&1 || { tail -40 $O/c25_tests.txt; exit 1; }
tail -1 $O/c25_tests.txt
timeout -k 10 120 python scripts/stem_pool_iso.py 2>&1 | grep -v amdgpu.ids | tee $O/c25_iso.txt
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --kernel-trace --pmc SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_WAIT_ANY -d $O/c25_pmc -o p --output-format csv -- \
  python3 $ROOT/scripts/stem_pool_iso.py --batch 32 > $O/c25_pmc.log 2>&1 || { tail -5 $O/c25_pmc.log; exit 1; }
python3 - <<'PY'
import csv, collections, glob
f = glob.glob("/root/repo/gpurun_out/r6/c25_pmc/**/*counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"].split("(")[0][-40:]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, c in agg.items():
    print(k, {kk: f"{v:.3g}" for kk, v in c.items()})
PY
