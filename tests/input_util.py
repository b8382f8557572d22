"""Seeded synthetic decoded images (HxWx3 uint8) shared by the input-pipeline fixtures
(tests/golden/gen_golden_input.py) and tests: numpy PCG64, platform-stable."""
import numpy as np

# (name, h, w, out_h, out_w, seed, kind, grayscale) -- the recorded Pillow cases
CASES = [
    ("cub_land", 375, 500, 224, 224, 1, "smooth", False),     # CUB-200 photo shapes -> 224
    ("cub_port", 500, 375, 224, 224, 2, "noise", False),
    ("cub_gray", 333, 500, 224, 224, 3, "smooth", True),      # get_grayscale (util/data.py:568-574)
    ("up_64", 64, 64, 96, 96, 4, "noise", False),             # upscale both axes
    ("up_mixed", 100, 150, 120, 90, 5, "smooth", False),      # up one axis, down the other
    ("shapes_128", 256, 256, 128, 128, 6, "smooth", False),   # geometric-shapes 128 (C5)
    ("shapes_64", 200, 300, 64, 64, 7, "noise", False),       # geometric-shapes 64 (C1)
    ("identity", 80, 60, 80, 60, 8, "noise", False),          # no resample pass
    ("h_only", 50, 200, 50, 64, 9, "noise", False),           # horizontal pass only
    ("v_only", 200, 50, 64, 50, 10, "noise", False),          # vertical pass only
    ("one_px", 1, 1, 5, 7, 11, "noise", False),
    ("row", 1, 500, 32, 32, 12, "noise", False),
    ("col", 500, 1, 32, 32, 13, "noise", True),
    ("tall_vfirst", 1000, 3, 64, 64, 14, "noise", False),     # Pillow's vertical-first branch
    ("tall_hfirst", 297, 2, 298, 40, 15, "noise", False),     # h > 100 w but upscaled: H first
    ("wide", 3, 1000, 64, 64, 16, "noise", False),
    ("odd", 37, 41, 40, 39, 17, "noise", False),
    ("tiny_up", 7, 5, 64, 64, 18, "smooth", False),
    ("big_down", 1500, 2000, 48, 64, 19, "smooth", False),     # 31x downscale, 63-tap rows
]


def synth_photo(h: int, w: int, seed: int, kind: str = "noise") -> np.ndarray:
    rng = np.random.Generator(np.random.PCG64(seed))
    if kind == "noise":
        return rng.integers(0, 256, size=(h, w, 3), dtype=np.uint8)
    yy, xx = np.meshgrid(np.linspace(0, 1, h), np.linspace(0, 1, w), indexing="ij")
    img = np.zeros((h, w, 3))
    for c in range(3):
        a, b, f, g, ph = rng.uniform(-1, 1, 5)
        img[..., c] = 128 + 90 * np.sin(2 * np.pi * (f * 3 * xx + g * 3 * yy) + ph) + 30 * (a * xx + b * yy)
    img += rng.normal(0, 12, size=img.shape)
    return np.clip(np.rint(img), 0, 255).astype(np.uint8)
