import torch, sys
from distributed_resnet_tensorflow_amd.models.spec import cifar_resnet_v2, imagenet_resnet_v2
from distributed_resnet_tensorflow_amd.ops.backend import HipBackend, RefBackend
from distributed_resnet_tensorflow_amd.runtime.executor import Executor
def rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return (a - b).norm().item() / max(b.norm().item(), 1e-12)
for spec, N in [(imagenet_resnet_v2(18, num_classes=10, image_size=64), 8), (imagenet_resnet_v2(18, num_classes=10, image_size=128), 32)]:
    torch.manual_seed(0)
    imgs = torch.randn(N, spec.image_size, spec.image_size, 3).bfloat16().float()
    labels = torch.randint(0, spec.num_classes, (N,), dtype=torch.int32)
    exs = {}
    for be, dev in ((RefBackend(), "cpu"), (HipBackend(), "cuda")):
        ex = Executor(spec, N, be, dev, seed=5)
        ex.P.master.copy_(ex.P.master.bfloat16().float()); ex.sync_weights()
        ex.images.zero_(); ex.images[..., :3] = imgs.to(dev); ex.labels.copy_(labels.to(dev))
        ex.forward(train=True); ex.backward(); exs[dev] = ex
    torch.cuda.synchronize()
    r, h = exs["cpu"], exs["cuda"]
    print(spec.name, N, 'logits', rel(h.logits, r.logits), 'stem_out', rel(h.stem_out, r.stem_out), 'pool', rel(h.pool_out, r.pool_out))
    for bp_h, bp_r in zip(h.blocks, r.blocks):
        print('  block out', rel(bp_h.out, bp_r.out))
    for s in h.P.slots:
        print('  ', s.name, round(rel(h.P.g(s.name), r.P.g(s.name)), 4))
