#!/usr/bin/env python3
"""Host input rate of the ImageNet pipeline (data/imagenet.py ImagenetLoader): JPEG decode +
packing of fake 500x375 JPEGs (the ImageNet median size, quality 90) in img/s, for 1..N decode
threads, and the per-core decode rate alone -- the number that says how many host cores one
MI355X needs at the trained step rate (reference: 5 parallel map threads + prefetch,
resnet_imagenet_main.py:158-183; VGG geometry vgg_preprocessing.py:284-333, which here runs on
the GPU).

    python scripts/imagenet_input_bench.py [--images 512] [--threads 1,2,4,8] [--workers thread,process]
Prints one JSON line per configuration.
"""
import argparse
import io
import json
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from distributed_resnet_tensorflow_amd.data import imagenet as inet  # noqa: E402
from distributed_resnet_tensorflow_amd.utils.tfrecord import TFRecordWriter  # noqa: E402


def natural_jpeg(rng, h=375, w=500):
    """A smooth, photo-like image (random smooth field + texture): decodes at a realistic cost
    (white noise JPEGs decode far slower than photographs)."""
    from PIL import Image
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float32)
    img = np.zeros((h, w, 3), np.float32)
    for c in range(3):
        for _ in range(4):
            fy, fx, ph = rng.uniform(0.002, 0.05), rng.uniform(0.002, 0.05), rng.uniform(0, 6.28)
            img[..., c] += np.sin(yy * fy + xx * fx + ph) * rng.uniform(20, 60)
    img += rng.normal(0, 8, img.shape)
    img = np.clip(img + 128, 0, 255).astype(np.uint8)
    b = io.BytesIO()
    Image.fromarray(img).save(b, format="JPEG", quality=90)
    return b.getvalue()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--images", type=int, default=512)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--threads", default="1,2,4,8")
    ap.add_argument("--workers", default="thread,process")
    args = ap.parse_args()
    rng = np.random.default_rng(0)
    d = tempfile.mkdtemp(prefix="drn_inbench_")
    protos = [natural_jpeg(rng) for _ in range(16)]
    per_shard = args.images // 2
    for s in range(2):
        with TFRecordWriter(os.path.join(d, "train-%05d-of-01024" % s)) as w:
            for i in range(per_shard):
                w.write(inet.make_example(protos[(s * per_shard + i) % len(protos)], 1 + i % 1000))
    # decode alone, one core
    t0 = time.perf_counter()
    n = 0
    while time.perf_counter() - t0 < 2.0:
        inet.decode_image(protos[n % len(protos)])
        n += 1
    per_core = n / (time.perf_counter() - t0)
    print(json.dumps({"what": "decode_one_core", "jpeg": "500x375 q90", "img_per_s": round(per_core, 1)}), flush=True)
    for workers in args.workers.split(","):
        for nt in [int(t) for t in args.threads.split(",")]:
            ld = inet.ImagenetLoader(d, args.batch, True, num_threads=nt, prefetch=3, num_epochs=None,
                                     workers=workers)
            next(ld)  # warm-up batch (process workers start here)
            t0 = time.perf_counter()
            nb = max(2, args.images // args.batch)
            for _ in range(nb):
                next(ld)
            dt = time.perf_counter() - t0
            ld.close()
            print(json.dumps({"what": "loader", "workers": workers, "n": nt, "batch": args.batch,
                              "img_per_s": round(nb * args.batch / dt, 1), "cpus": os.cpu_count()}), flush=True)


if __name__ == "__main__":
    main()
