# round-6 GPU call 7: interleaved A/B of the step-level changes on one box (shipped database):
# HW queues 8 vs 4, in-kernel wgrad split-K reduction on/off, CU-masked weight-gradient stream
set -o pipefail
mkdir -p gpurun_out/r6
OUT=gpurun_out/r6/ab7.jsonl
: > $OUT
for round in 1 2; do
  for arm in base hwq4 fusedonly cu128 cu192 cu64; do
    case $arm in
      base) env="" ;;
      hwq4) env="GPU_MAX_HW_QUEUES=4" ;;
      fusedonly) env="DRN_WGRAD_MODES=2" ;;
      cu128) env="DRN_SIDE_CUS=128" ;;
      cu192) env="DRN_SIDE_CUS=192" ;;
      cu64) env="DRN_SIDE_CUS=64" ;;
    esac
    line=$(env $env timeout -k 10 300 python bench.py 2>> gpurun_out/r6/ab7.err) || { echo "arm $arm failed"; tail -5 gpurun_out/r6/ab7.err; exit 1; }
    echo "{\"arm\": \"$arm\", \"round\": $round, \"r\": $line}" >> $OUT
    echo "$arm $round $(echo $line | cut -c1-160)"
  done
done
