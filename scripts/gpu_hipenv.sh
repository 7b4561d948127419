#!/bin/bash
# HIP runtime launch knobs (process environment): graph packet capture, device kernargs.
OUT=${1:-gpurun_out/hipenv}
export PYTHONPATH=$(pwd)
mkdir -p "$OUT"
for r in 1 2; do
  for v in "base=X=1" "devka=HIP_FORCE_DEV_KERNARG=1" "pcap=DEBUG_CLR_GRAPH_PACKET_CAPTURE=1" "both=HIP_FORCE_DEV_KERNARG=1 DEBUG_CLR_GRAPH_PACKET_CAPTURE=1"; do
    name=${v%%=*}; envs=${v#*=}
    for bs in 32 128; do
      line=$(env $envs timeout -k 10 200 python bench.py --dataset cifar10 --batch_size $bs --steps 50 --warmup 10 2>> "$OUT/err.txt") || { tail "$OUT/err.txt"; exit 1; }
      echo "$r $name cifar$bs $(echo "$line" | python3 -c 'import sys,json; print(json.loads(sys.stdin.read())["ms_per_step"])')" | tee -a "$OUT/ab.txt"
    done
    line=$(env $envs timeout -k 10 200 python bench.py 2>> "$OUT/err.txt") || { tail "$OUT/err.txt"; exit 1; }
    echo "$r $name rn50 $(echo "$line" | python3 -c 'import sys,json; print(json.loads(sys.stdin.read())["ms_per_step"])')" | tee -a "$OUT/ab.txt"
  done
done
