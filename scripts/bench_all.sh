export PYTHONPATH=$(pwd)
O=gpurun_out/b13; mkdir -p $O
timeout -k 10 240 python bench.py --steps 50 --warmup 10 > $O/rn50.json 2> $O/rn50.err && \
timeout -k 10 240 python bench.py --dataset cifar10 --steps 200 --warmup 20 > $O/cifar.json 2> $O/cifar.err && \
timeout -k 10 300 python bench.py --width 2 --batch_size 256 --steps 20 --warmup 5 > $O/wrn.json 2> $O/wrn.err && \
cat $O/*.json
