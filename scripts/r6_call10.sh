# round-6 GPU call 10: occupancy cap of the weight-gradient side stream in the replayed plan
# (DRN_SIDE_LDS_MIN_KB: every side-stream launch requests at least that much LDS), interleaved A/B
set -o pipefail
mkdir -p gpurun_out/r6
OUT=gpurun_out/r6/ab10.jsonl
: > $OUT
for round in 1 2 3; do
  for kb in 0 84 56 100; do
    line=$(DRN_SIDE_LDS_MIN_KB=$kb timeout -k 10 300 python bench.py --plan 1 2>> gpurun_out/r6/ab10.err) || { echo "arm $kb failed"; tail -5 gpurun_out/r6/ab10.err; exit 1; }
    echo "{\"side_lds_kb\": $kb, \"round\": $round, \"r\": $line}" >> $OUT
    echo "$kb $round $(echo $line | cut -c100-200)"
  done
done
