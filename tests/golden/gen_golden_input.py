"""Record Pillow's outputs for the evaluation input transform (tests/golden/input_resize.npz).

The reference's transform_no_augment (util/data.py:264-269, :500-505, ...) resizes PIL images
with torchvision's Resize, which forwards to ``PIL.Image.resize(size[::-1], BILINEAR)``;
torchvision itself is absent here, so this records what it would call: Pillow (12.2.0 in this
image) on seeded synthetic images (tests/input_util.py), plus ``convert('L')`` for the
Grayscale(3) cases.  Stored per case: the resized uint8 HxWx3 image (inputs are regenerated
from their seeds).

Usage:  python tests/golden/gen_golden_input.py
"""
import os
import sys

import numpy as np
from PIL import Image

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from input_util import CASES, synth_photo  # noqa: E402


def main():
    import PIL
    out = {"pillow_version": np.array(PIL.__version__)}
    for name, h, w, oh, ow, seed, kind, gray in CASES:
        img = Image.fromarray(synth_photo(h, w, seed, kind), "RGB")
        r = img.resize((ow, oh), Image.BILINEAR)
        if gray:      # torchvision F_pil.to_grayscale(img, 3): convert('L') stacked 3x
            l = np.asarray(r.convert("L"))
            arr = np.dstack([l, l, l])
        else:
            arr = np.asarray(r)
        out[name] = np.ascontiguousarray(arr, dtype=np.uint8)
    path = os.path.join(HERE, "input_resize.npz")
    np.savez_compressed(path, **out)
    print(path, os.path.getsize(path), "bytes,", len(CASES), "cases")


if __name__ == "__main__":
    main()
