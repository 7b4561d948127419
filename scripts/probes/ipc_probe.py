"""Probe HIP IPC handle export/open between two processes on one GPU (debug helper)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))  # repo root
import torch
import torch.multiprocessing as mp

from distributed_resnet_tensorflow_amd.parallel.p2p import _IpcHandle, _export, _hip


def child(q, r):
    torch.cuda.set_device(0)
    torch.zeros(1, device="cuda")
    hb, off = q.get()
    h = _hip()
    for flags in (0, 1):
        hd = _IpcHandle.from_bytes(hb)
        p = ctypes.c_void_p()
        rc = h.hipIpcOpenMemHandle(ctypes.byref(p), hd, flags)
        print("open flags", flags, "rc", rc, "ptr", p.value, flush=True)
        if rc == 0:
            t = torch.empty(4, device="cuda")
            # read the first 4 floats through a raw device-to-device copy
            h.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
            print("memcpy rc", h.hipMemcpy(ctypes.c_void_p(t.data_ptr()), ctypes.c_void_p(p.value + off), 16, 3),
                  t.cpu().tolist(), flush=True)
            h.hipIpcCloseMemHandle(p)
    r.put(1)


if __name__ == "__main__":
    torch.cuda.set_device(0)
    x = torch.arange(1024, dtype=torch.float32, device="cuda") + 7
    ctx = mp.get_context("spawn")
    q, r = ctx.Queue(), ctx.Queue()
    p = ctx.Process(target=child, args=(q, r))
    p.start()
    hb, off = _export(x)
    print("exported offset", off, "handle head", hb[:16].hex(), flush=True)
    q.put((hb, off))
    r.get(timeout=120)
    p.join(timeout=60)
    # the same through torch's own CUDA IPC (ForkingPickler) for comparison
    def torch_child(q2, r2):
        t = q2.get()
        print("torch-ipc read", t[:4].cpu().tolist(), flush=True)
        r2.put(1)
