"""Diagnostic: CIFAR GPU feeder with pinned loader batches, stack dumps if it stalls."""
import faulthandler
import sys
import tempfile
import time

sys.path.insert(0, ".")
faulthandler.dump_traceback_later(30, repeat=True, file=sys.stderr)
import numpy as np
import torch

from distributed_resnet_tensorflow_amd.data import cifar
from distributed_resnet_tensorflow_amd.models.spec import cifar_resnet_v2
from distributed_resnet_tensorflow_amd.ops.backend import HipBackend
from distributed_resnet_tensorflow_amd.runtime.executor import Executor
from distributed_resnet_tensorflow_amd.train.feeder import CifarFeeder

d = tempfile.mkdtemp()
cifar.write_fake_cifar(d, 120)
rec = cifar.CifarRecords(cifar.get_filenames(True, d))
t0 = time.time()
ld = cifar.CifarLoader(rec, 64, True, seed=4, pin=True, pin_device=torch.device("cuda"))
print("loader up", time.time() - t0, flush=True)
b = next(ld)
print("first batch", type(b[0]), b[0].is_pinned(), time.time() - t0, flush=True)
ex = Executor(cifar_resnet_v2(8), 64, HipBackend(), "cuda")
print("executor", time.time() - t0, flush=True)
f = CifarFeeder(ex, ld, True)
for k in range(10):
    f.next()
    print("step", k, time.time() - t0, flush=True)
torch.cuda.synchronize()
f.close()
print("done", flush=True)
