#!/bin/bash
# Tests of the split finalize / trial paths, then step A/Bs: split finalize on/off, claim query,
# cold tuner; then a kernel-trace profile of the default step.
OUT=${1:-gpurun_out/ab4}
export PYTHONPATH=$(pwd)
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py tests/test_executor_gpu.py tests/test_dp_gpu.py -x -q --timeout 300 \
  --timeout-method thread -k "finalize or non_publishing or executor or times_eager" > "$OUT/tests.log" 2>&1
rc=$?; tail -3 "$OUT/tests.log"; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" "$OUT/tests.log" | head -20; exit $rc; }
timeout -k 10 300 python scripts/host_vs_gpu.py > "$OUT/host_vs_gpu.txt" 2> "$OUT/host_vs_gpu.err" || { tail "$OUT/host_vs_gpu.err"; exit 1; }
cat "$OUT/host_vs_gpu.txt"
bash scripts/gpu_env_ab.sh "$OUT" ${ROUNDS:-2} "base=DRN_BN_FIN_SPLIT_C=100000 DRN_CFIN_MAX_WORK=1000000000000 DRN_CLAIM_QUERY=0" \
  "new=DRN_CLAIM_QUERY=1" "late=DRN_WGRAD_LATE=1" "cold=DRN_TUNE_COLD=1" || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/$OUT/prof" -o step -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 3 > "$GRAFT_REPO_ROOT/$OUT/prof.log" 2>&1 || { tail "$GRAFT_REPO_ROOT/$OUT/prof.log"; exit 1; }
python3 "$GRAFT_REPO_ROOT/scripts/step_streams.py" "$GRAFT_REPO_ROOT/$OUT/prof/step_kernel_trace.csv" > "$GRAFT_REPO_ROOT/$OUT/streams.txt"
head -12 "$GRAFT_REPO_ROOT/$OUT/streams.txt"
