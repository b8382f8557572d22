"""Evaluation input transform: GPU (pipnet_resize_normalize_rgb8) vs the reference's host path.

The reference runs transform_no_augment (util/data.py:500-505: Resize((224,224)) + ToTensor +
Normalize) per image in DataLoader workers.  Workload: a CUB-200-shaped batch of 64 decoded
RGB photos (sizes uniform in 200..500 px, seeded), output [64,3,224,224] fp32.
Prints one JSON line:
  gpu_kernel_*   : the launch alone (inputs resident in HBM), HIP events on the launching stream;
  gpu_h2d_*      : packed uint8 batch host(pinned) -> device + launch;
  cpu_ref_*      : Pillow resize + torch ToTensor/Normalize (the reference's ops), 1 core;
  jpeg_decode_*  : Pillow JPEG decode of the same photos (what stays on the host), 1 core.
    python tools/bench_input.py [--batch 64] [--reps 50]
"""
import argparse
import io
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from count_pipnet_amd import build  # noqa: E402
from count_pipnet_amd import kernels as K  # noqa: E402
from count_pipnet_amd.data import IMAGENET_MEAN, IMAGENET_STD, pack_images  # noqa: E402
from input_util import synth_photo  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--size", type=int, default=224)
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    build.build()
    torch.set_num_threads(1)
    rng = np.random.default_rng(0)
    imgs = [synth_photo(int(h), int(w), 100 + i, "smooth") for i, (h, w) in enumerate(rng.integers(200, 501, (a.batch, 2)))]
    packed = pack_images(imgs)
    res = {"batch": a.batch, "out": [3, a.size, a.size], "mean_in_px": float(np.mean([im.shape[0] * im.shape[1] for im in imgs]))}
    in_bytes = int(sum(im.size for im in imgs))
    out_bytes = a.batch * 3 * a.size * a.size * 4
    res["algorithmic_bytes"] = in_bytes + out_bytes
    if torch.cuda.is_available():
        dev = torch.device("cuda:0")
        pin = packed.pixels.pin_memory()
        pix = pin.to(dev)
        off = packed.offsets.to(dev)
        siz = packed.sizes.to(dev)
        sh = packed.sizes.numpy()
        run = lambda p: K.resize_normalize_rgb8(p, off, siz, sh, (a.size, a.size), IMAGENET_MEAN, IMAGENET_STD)
        for _ in range(5):
            run(pix)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            run(pix)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.reps
        res["gpu_kernel_ms_per_batch"] = ms
        res["gpu_kernel_images_per_sec"] = a.batch / ms * 1e3
        res["gpu_kernel_GBps"] = res["algorithmic_bytes"] / ms / 1e6
        e0.record()
        for _ in range(a.reps):
            run(pin.to(dev, non_blocking=True))
        e1.record()
        torch.cuda.synchronize()
        ms2 = e0.elapsed_time(e1) / a.reps
        res["gpu_h2d_ms_per_batch"] = ms2
        res["gpu_h2d_images_per_sec"] = a.batch / ms2 * 1e3
    from PIL import Image

    from oracle.input_ref import to_tensor_normalize
    pil = [Image.fromarray(im, "RGB") for im in imgs]
    t0 = time.perf_counter()
    n = 0
    while time.perf_counter() - t0 < 3.0:
        for im in pil:
            r = im.resize((a.size, a.size), Image.BILINEAR)
            to_tensor_normalize(np.asarray(r))
            n += 1
    dt = time.perf_counter() - t0
    res["cpu_ref_images_per_sec_1core"] = n / dt
    jpgs = []
    for im in pil[:16]:
        b = io.BytesIO()
        im.save(b, "JPEG", quality=90)
        jpgs.append(b.getvalue())
    t0 = time.perf_counter()
    n = 0
    while time.perf_counter() - t0 < 2.0:
        for j in jpgs:
            np.asarray(Image.open(io.BytesIO(j)).convert("RGB"))
            n += 1
    res["jpeg_decode_images_per_sec_1core"] = n / (time.perf_counter() - t0)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
