"""drn: MI355X-native distributed ResNet training (see README.md)."""
# Hardware queues: the package keeps HIP's default (GPU_MAX_HW_QUEUES=4 normal-priority queues
# per process) and instead keeps the number of busy normal-priority streams within it (the
# ImageNet feeder's H2D copy stream is high-priority: train/feeder.py). Raising the queue count
# was measured and rejected: with 5, 6 or 8 queues some multi-stream step modes fall into 3-5x
# slower steps (queues time-sliced, kernels and cross-queue waits stretched: CIFAR ResNet-50 bs32
# whole-step graph 4.7-6.3 ms and P2P native plan 8.6-9.4 ms vs 1.8-1.9 ms with 4 queues,
# profiles/r6_p2p_plan_queues.txt).
