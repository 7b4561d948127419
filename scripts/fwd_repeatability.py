"""Repeated training-mode forwards from one state (nondeterministic mode): which block output
changes between repetitions, and by how much (BN-statistics atomics + amplification).

    python scripts/fwd_repeatability.py [batch] [image_size]
"""
import sys
import torch
from distributed_resnet_tensorflow_amd.models.spec import imagenet_resnet_v2
from distributed_resnet_tensorflow_amd.ops.backend import HipBackend
from distributed_resnet_tensorflow_amd.runtime.executor import Executor

N = int(sys.argv[1]) if len(sys.argv) > 1 else 4
size = int(sys.argv[2]) if len(sys.argv) > 2 else 64
be = HipBackend("cuda")
ex = Executor(imagenet_resnet_v2(50, num_classes=11, image_size=size), N, be, "cuda", seed=5, weight_decay=1e-4)
be.synthetic_images(ex.images, seed=9)
ex.labels.copy_(torch.arange(N, dtype=torch.int32) % 11)
ex.set_lr(0.02)
ex.autotune()
torch.cuda.synchronize()


def snap():
    outs = [ex.stem_out, ex.pool_out] + [bp.out for bp in ex.blocks] + [ex.logits]
    return [o.float().clone() for o in outs]


ref = None
for rep in range(12):
    ex.forward(train=True)
    torch.cuda.synchronize()
    s = snap()
    loss = float(ex.loss_vec.float().mean())
    if ref is None:
        ref = s
        print(f"rep 0 loss {loss:.6f}")
        continue
    dev = [float((a - b).abs().max() / (b.abs().max() + 1e-30)) for a, b in zip(s, ref)]
    first = next((i for i, d in enumerate(dev) if d > 1e-2), None)
    print(f"rep {rep} loss {loss:.6f} first deviating output {first} max rel dev {max(dev):.3e} "
          f"per-output {' '.join(f'{d:.1e}' for d in dev)}", flush=True)
