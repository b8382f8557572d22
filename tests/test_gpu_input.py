"""Evaluation input transform on the GPU (pipnet_resize_normalize_rgb8 through the C-ABI)
against the oracle restatement and Pillow's recorded outputs (tests/golden/input_resize.npz):
bit-exact -- the resize is integer arithmetic and ToTensor/Normalize are IEEE fp32 ops."""
import os

import numpy as np
import pytest
import torch

from input_util import CASES, synth_photo
from oracle import input_ref

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "input_resize.npz")


def _run(gpu, images, size, gray=False):
    from count_pipnet_amd.data import DeviceEvalTransform, pack_images
    out, u8 = DeviceEvalTransform(size, grayscale=gray)(pack_images(images), gpu, want_u8=True)
    torch.cuda.synchronize()
    return out.cpu(), u8.cpu().numpy()


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_resize_normalize_vs_pillow_golden(gpu, case):
    name, h, w, oh, ow, seed, kind, gray = case
    g = np.load(GOLDEN)[name]
    out, u8 = _run(gpu, [synth_photo(h, w, seed, kind)], (oh, ow), gray)
    np.testing.assert_array_equal(u8[0], g)
    assert torch.equal(out[0], input_ref.to_tensor_normalize(g))


def test_ragged_batch_all_cases_one_launch(gpu):
    """Every golden case resized to one common size in ONE launch (ragged input batch)."""
    imgs = [synth_photo(h, w, seed, kind) for _, h, w, _, _, seed, kind, _ in CASES]
    out, u8 = _run(gpu, imgs, (57, 83))
    for i, im in enumerate(imgs):
        t, r = input_ref.eval_transform(im, (57, 83))
        np.testing.assert_array_equal(u8[i], r, err_msg=CASES[i][0])
        assert torch.equal(out[i], t), CASES[i][0]


def test_cub_batch_224(gpu):
    """A CUB-200-shaped evaluation batch (bs=64, photo sizes 200..500 px) -> 224x224."""
    rng = np.random.default_rng(7)
    imgs = [synth_photo(int(h), int(w), 500 + i, "smooth" if i % 2 else "noise")
            for i, (h, w) in enumerate(rng.integers(200, 501, (64, 2)))]
    out, u8 = _run(gpu, imgs, 224)
    assert out.shape == (64, 3, 224, 224)
    for i in range(0, 64, 7):
        t, r = input_ref.eval_transform(imgs[i], (224, 224))
        np.testing.assert_array_equal(u8[i], r)
        assert torch.equal(out[i], t)


def test_device_loader_end_to_end(gpu, tmp_path):
    """ImageFolder on disk (lossless PNG) -> DeviceEvalLoader -> the reference transform."""
    from PIL import Image

    from count_pipnet_amd.data import DecodedImageFolder, DeviceEvalLoader, DeviceEvalTransform
    want = {}
    for c in range(3):
        os.makedirs(tmp_path / f"class_{c}")
        for j in range(3):
            im = synth_photo(40 + 13 * j, 60 + 7 * c, 10 * c + j, "smooth")
            p = str(tmp_path / f"class_{c}" / f"img{j}.png")
            Image.fromarray(im, "RGB").save(p)
            want[p] = (im, c)
    ds = DecodedImageFolder(str(tmp_path))
    loader = DeviceEvalLoader(ds, DeviceEvalTransform(32), gpu, batch_size=4, num_workers=0, shuffle=False)
    assert len(loader) == 3
    seen = 0
    for xs, ys in loader:
        assert xs.is_cuda and xs.dtype == torch.float32 and ys.is_cuda and ys.dtype == torch.int64
        for k in range(xs.shape[0]):
            path, cls = ds.samples[seen]
            im, c = want[path]
            assert int(ys[k]) == c == cls
            assert torch.equal(xs[k].cpu(), input_ref.eval_transform(im, (32, 32))[0])
            seen += 1
    assert seen == 9


def test_empty_batch_and_errors(gpu):
    from count_pipnet_amd import kernels as K
    from count_pipnet_amd.data import DeviceEvalTransform, pack_images
    out = DeviceEvalTransform(16)(pack_images([]), gpu)
    assert out.shape == (0, 3, 16, 16)
    with pytest.raises(RuntimeError):
        K.resize_normalize_rgb8(torch.zeros(4, device=gpu), torch.zeros(1, dtype=torch.int64, device=gpu),
                                torch.ones(1, 2, dtype=torch.int32, device=gpu), [[1, 1]], (4, 4),
                                input_ref.IMAGENET_MEAN, input_ref.IMAGENET_STD)
