#!/usr/bin/env python3
"""Host throughput of the real-data ImageNet input pipeline (no GPU needed).

Writes one synthetic TFRecord shard of JPEGs (ImageNet-like 500x375 photos-ish:
smooth colour fields + texture, quality 90, 1-based labels) and times
data/imagenet.input_fn over it:
  float : the reference-equivalent CPU VGG pipeline (decode, resize, crop, flip,
          mean subtraction) -> float32 NHWC (4 B / value to the device)
  u8    : decode, resize, crop -> uint8 NHWC (1 B / value); flip + mean + bf16
          packing run on the device (imagenet_u8_pack)

  python scripts/imagenet_loader_bench.py [n_images] [workers ...]
"""
import io
import os
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_tensorflow_resnet_amd.data import imagenet  # noqa: E402
from distributed_tensorflow_resnet_amd.utils import records  # noqa: E402


def write_shard(path, n, seed=0):
    from PIL import Image

    rng = np.random.default_rng(seed)
    w = records.RecordWriter(path)
    for i in range(n):
        h, wd = (375, 500) if i % 3 else (500, 375)
        base = rng.integers(0, 256, (h // 25 + 1, wd // 25 + 1, 3)).astype(np.uint8)
        img = Image.fromarray(base).resize((wd, h), Image.BILINEAR)
        arr = np.asarray(img, dtype=np.int16) + rng.integers(-20, 21, (h, wd, 3))
        buf = io.BytesIO()
        Image.fromarray(np.clip(arr, 0, 255).astype(np.uint8)).save(buf, format="JPEG", quality=90)
        w.write(records.make_example({"image/encoded": buf.getvalue(), "image/format": b"JPEG",
                                      "image/class/label": int(rng.integers(1, 1001))}))
    w.close()


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 768
    workers = [int(a) for a in sys.argv[2:]] or [1, 4, 8]
    d = tempfile.mkdtemp()
    shards = max(workers)   # workers split the shard list (resnet_imagenet_main.py:166-192)
    for k in range(shards):
        write_shard(os.path.join(d, "train-%05d-of-01024" % k), n // shards, seed=k)
    mb = sum(os.path.getsize(os.path.join(d, f)) for f in os.listdir(d)) / 2 ** 20
    print(f"{shards} shards: {n} JPEGs, {mb:.1f} MiB; host CPUs {os.cpu_count()}")
    print("| path | workers | img/s | batch bytes to device |")
    print("|---|---|---|---|")
    for u8 in (False, True):
        for wk in workers:
            # the whole pass incl. worker start-up (the shuffle buffer holds up to 1024
            # records, so the first batch waits for most of a small shard anyway)
            it = imagenet.input_fn(True, d, 64, num_epochs=1, workers=wk, u8=u8)
            t0, cnt, first = time.perf_counter(), 0, None
            for x, y in it:
                first = x if first is None else first
                cnt += x.shape[0]
            dt = time.perf_counter() - t0
            print(f"| {'u8' if u8 else 'float'} | {wk} | {cnt / dt:.0f} | "
                  f"{first.numel() * first.element_size() / 2 ** 20:.1f} MiB / 64 img |", flush=True)


if __name__ == "__main__":
    main()
