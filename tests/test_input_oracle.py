"""Evaluation input transform, CPU side: the oracle's restatement of
Pillow's BILINEAR resample is pinned against Pillow's own outputs (tests/golden/input_resize.npz,
tests/golden/gen_golden_input.py), the ImageFolder semantics of count_pipnet_amd.data, and the
host-only planning entry point of the C-ABI (no GPU here)."""
import ctypes
import os

import numpy as np
import pytest
import torch

from input_util import CASES, synth_photo
from oracle import input_ref

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "input_resize.npz")


@pytest.fixture(scope="module")
def golden():
    return np.load(GOLDEN)


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_oracle_matches_pillow_golden(golden, case):
    name, h, w, oh, ow, seed, kind, gray = case
    _, r = input_ref.eval_transform(synth_photo(h, w, seed, kind), (oh, ow), grayscale=gray)
    assert r.shape == (oh, ow, 3)
    np.testing.assert_array_equal(r, golden[name])


def test_oracle_matches_pillow_random_sizes():
    """Against the Pillow in this image directly, on random sizes (incl. tall / wide)."""
    Image = pytest.importorskip("PIL.Image")
    rng = np.random.default_rng(123)
    sizes = [tuple(int(v) for v in s) for s in rng.integers(1, 300, (40, 4))]
    sizes += [(900, 4, 50, 70), (400, 4, 401, 30), (401, 4, 400, 30), (4, 900, 50, 70)]
    for i, (h, w, oh, ow) in enumerate(sizes):
        img = synth_photo(h, w, 1000 + i, "noise")
        ref = np.asarray(Image.fromarray(img, "RGB").resize((ow, oh), Image.BILINEAR))
        np.testing.assert_array_equal(input_ref.pil_resize_bilinear(img, oh, ow), ref, err_msg=str((h, w, oh, ow)))


def test_to_tensor_normalize_restatement():
    """ToTensor + Normalize (torchvision) as the reference applies them, fp32 on CPU."""
    img = synth_photo(9, 11, 5)
    t = input_ref.to_tensor_normalize(img)
    x = torch.from_numpy(img).permute(2, 0, 1).float() / 255.0
    ref = (x - torch.tensor(input_ref.IMAGENET_MEAN)[:, None, None]) / torch.tensor(input_ref.IMAGENET_STD)[:, None, None]
    assert t.dtype == torch.float32 and t.shape == (3, 9, 11)
    assert torch.equal(t, ref)


def test_resize_plan_host_entry():
    from count_pipnet_amd import _lib
    lib = _lib.load()
    sizes = np.array([[375, 500], [1000, 3], [64, 64]], np.int32)
    kmax, ws = ctypes.c_int(0), ctypes.c_int64(0)
    assert lib.pipnet_resize_plan(sizes.ctypes.data, 3, 224, 224, ctypes.byref(kmax), ctypes.byref(ws)) == 0
    want = max(input_ref.precompute_coeffs(int(v), 224)[1].shape[1] for v in sizes.reshape(-1))
    assert kmax.value == want
    assert ws.value == 3 * (224 + 224) * (2 + want) * 4
    bad = np.array([[0, 5]], np.int32)
    assert lib.pipnet_resize_plan(bad.ctypes.data, 1, 224, 224, ctypes.byref(kmax), ctypes.byref(ws)) == 1
    assert lib.pipnet_resize_plan(sizes.ctypes.data, 3, 0, 224, ctypes.byref(kmax), ctypes.byref(ws)) == 1


def _write_tree(root, layout):
    from PIL import Image
    for cls, files in layout.items():
        os.makedirs(os.path.join(root, cls), exist_ok=True)
        for j, (fname, h, w) in enumerate(files):
            path = os.path.join(root, cls, fname)
            os.makedirs(os.path.dirname(path), exist_ok=True)
            if fname.endswith(".txt"):
                open(path, "w").write("not an image")
            else:
                Image.fromarray(synth_photo(h, w, hash((cls, fname)) % 1000, "smooth"), "RGB").save(path)


def test_image_folder_semantics(tmp_path):
    """torchvision ImageFolder: sorted classes, sorted walk (sub-folders too), extension filter."""
    from count_pipnet_amd.data import DecodedImageFolder
    _write_tree(tmp_path, {
        "b_cls": [("z.png", 10, 12), ("a.PNG", 8, 9), ("notes.txt", 0, 0), ("sub/c.png", 5, 5)],
        "a_cls": [("x.bmp", 6, 7)],
        "c_cls": [("y.png", 4, 4)],
    })
    ds = DecodedImageFolder(str(tmp_path))
    assert ds.classes == ["a_cls", "b_cls", "c_cls"]
    assert ds.class_to_idx == {"a_cls": 0, "b_cls": 1, "c_cls": 2}
    rel = [(os.path.relpath(p, tmp_path), t) for p, t in ds.samples]
    assert rel == [("a_cls/x.bmp", 0), ("b_cls/a.PNG", 1), ("b_cls/z.png", 1), ("b_cls/sub/c.png", 1),
                   ("c_cls/y.png", 2)]
    assert ds.targets == [0, 1, 1, 1, 2]
    img, t = ds[2]
    assert img.dtype == np.uint8 and img.shape == (10, 12, 3) and t == 1


def test_image_folder_errors(tmp_path):
    from count_pipnet_amd.data import DecodedImageFolder
    with pytest.raises(FileNotFoundError):
        DecodedImageFolder(str(tmp_path))                       # no class folders
    _write_tree(tmp_path, {"a": [("x.png", 3, 3)], "empty": [("n.txt", 0, 0)]})
    with pytest.raises(FileNotFoundError, match="empty"):
        DecodedImageFolder(str(tmp_path))                       # class without a valid file


def test_pack_images_layout():
    from count_pipnet_amd.data import pack_images
    ims = [synth_photo(3, 4, 1), synth_photo(5, 2, 2), synth_photo(1, 1, 3)]
    p = pack_images(ims, [7, 8, 9])
    assert p.offsets.tolist() == [0, 36, 66]
    assert p.sizes.tolist() == [[3, 4], [5, 2], [1, 1]]
    assert p.targets.tolist() == [7, 8, 9]
    flat = p.pixels.numpy()
    for im, o in zip(ims, p.offsets.tolist()):
        np.testing.assert_array_equal(flat[o:o + im.size].reshape(im.shape), im)
    with pytest.raises(ValueError):
        pack_images([np.zeros((2, 2), np.uint8)])


def test_device_transform_refuses_cpu():
    from count_pipnet_amd.data import DeviceEvalTransform, pack_images
    with pytest.raises(RuntimeError, match="ROCm"):
        DeviceEvalTransform(8)(pack_images([synth_photo(4, 4, 1)]), "cpu")
