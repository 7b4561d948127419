# round-6 GPU call 21: where the P2P data-parallel step's +0.34 ms over the single-GPU step goes
# (CIFAR bs32, single-rank engine, 4 hardware queues): reduces inline on the compute stream, no
# error-word copy, both
set -o pipefail
ROOT=$(pwd)
O=$ROOT/gpurun_out/r6
mkdir -p $O
export PYTHONPATH=$ROOT
B="--dataset cifar10 --batch_size 32 --steps 100 --warmup 10"
for cfg in "base|1|1" "inline|1|0" "nocopy|0|1" "inline_nocopy|0|0" "base|1|1" "inline_nocopy|0|0"; do
  IFS='|' read name cp nl <<< "$cfg"
  inl=$((1-nl))
  DRN_P2P_INLINE=$inl DRN_P2P_ERR_COPY=$cp DRN_BENCH_DP=1 timeout -k 10 200 python bench.py $B --allreduce p2p > $O/c21_x.json 2>> $O/c21.err || { tail $O/c21.err; exit 1; }
  echo "$name $(grep -o '"ms_per_step": [0-9.]*\|"step_mode": "[a-z_]*"\|"mode_trial_ms": {[^}]*}' $O/c21_x.json | tr '\n' ' ')" | tee -a $O/c21_modes.txt
done
