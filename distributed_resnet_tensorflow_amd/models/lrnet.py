"""LRNet: the reference's one-hidden-layer MLP baseline (logist_model.py:14-86).

  x [B, S*S*3] -> xw_plus_b(hid_w [S*S*3, H], hid_b) -> ReLU -> xw_plus_b(sm_w [H,10], sm_b)
  -> softmax; loss = -sum(y * log(clip(p, 1e-10, 1))) (a SUM over the batch, not a mean);
  Adam(--learning_rate); hid_w ~ truncated_normal(stddev 1/S), sm_w ~ truncated_normal(1/sqrt(H)).
It is dead code on the reference's ResNet path (imported, unused: resnet_cifar_main.py:27); kept
for capability parity via `--model=lrnet`. It is tiny (<1 MFLOP/image), so it runs as plain
PyTorch autograd on any device, with the same data-parallel all-reduce (gradient average) when
distributed.
"""
from __future__ import annotations

import logging
import math

import torch

log = logging.getLogger("drn")


def _trunc(shape, std, gen):
    t = torch.randn(shape, generator=gen)
    t = torch.where(t.abs() > 2, torch.randn(shape, generator=gen).clamp(-2, 2), t)
    return t * std


class LRNet(torch.nn.Module):
    def __init__(self, image_size: int = 32, hidden_units: int = 100, num_classes: int = 10, seed: int = 0):
        super().__init__()
        g = torch.Generator().manual_seed(seed)
        d = image_size * image_size * 3
        self.hid_w = torch.nn.Parameter(_trunc((d, hidden_units), 1.0 / image_size, g))
        self.hid_b = torch.nn.Parameter(torch.zeros(hidden_units))
        self.sm_w = torch.nn.Parameter(_trunc((hidden_units, num_classes), 1.0 / math.sqrt(hidden_units), g))
        self.sm_b = torch.nn.Parameter(torch.zeros(num_classes))

    def forward(self, images_nhwc):
        x = images_nhwc[..., :3].reshape(images_nhwc.shape[0], -1).float()
        hid = torch.relu(x @ self.hid_w + self.hid_b)
        return torch.softmax(hid @ self.sm_w + self.sm_b, dim=1)

    @staticmethod
    def loss(pred, labels):
        y = torch.nn.functional.one_hot(labels.long(), pred.shape[1]).float()
        return -(y * torch.log(pred.clamp(1e-10, 1.0))).sum()


def train_lrnet(FLAGS, cluster):
    from ..parallel import cluster as cl
    from .spec import build_spec
    from ..ops.backend import RefBackend
    from ..runtime.executor import Executor
    from ..train.trainer import make_feeder
    cl.init_process_group(cluster)
    dev = torch.device(cluster.device)
    net = LRNet(FLAGS.image_size, FLAGS.hidden_units, 10, FLAGS.seed).to(dev)
    opt = torch.optim.Adam(net.parameters(), lr=FLAGS.learning_rate)
    # reuse the CIFAR pipeline (fp32 reference preprocessing) through a shim executor-like holder
    spec = build_spec("cifar10", 8)
    holder = Executor(spec, FLAGS.batch_size, RefBackend(), "cpu")
    feeder = make_feeder(FLAGS, holder, cluster, True)
    if cluster.distributed:
        import torch.distributed as dist
        for p in net.parameters():
            dist.broadcast(p.data, 0)
    step = 0
    try:
        while step < FLAGS.train_steps:
            feeder.next()
            imgs = holder.images.to(dev)
            pred = net(imgs)
            loss = LRNet.loss(pred, holder.labels.to(dev))
            opt.zero_grad()
            loss.backward()
            if cluster.distributed:
                import torch.distributed as dist
                for p in net.parameters():
                    dist.all_reduce(p.grad)
                    p.grad.div_(cluster.world)
            opt.step()
            step += 1
            if step % FLAGS.log_every_n_steps == 0:
                prec = (pred.argmax(1).cpu() == holder.labels.long()).float().mean().item()
                log.info("step = %d, loss = %.5f, precision = %.5f", step, loss.item(), prec)
    finally:
        feeder.close()
    return 0
