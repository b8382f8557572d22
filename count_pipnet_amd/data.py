"""Evaluation input pipeline -- drop-in for the reference's test loaders.

The reference builds every evaluation set as
``torchvision.datasets.ImageFolder(dir, transform=transform_no_augment)`` with
``transform_no_augment = Compose([Resize((s, s)), (Grayscale(3),) ToTensor(), normalize])``
(util/data.py:218-259 ``create_datasets``; transforms :264-269, :314-321, :500-505, :537-542,
:568-574) and iterates it through ``DataLoader(..., pin_memory=cuda, num_workers=...)``
(util/data.py:160-214), moving each ``(xs, ys)`` batch to the GPU in ``eval_pipnet``
(pipnet/test.py:67-69).  Per image the host decodes the file, resizes it (Pillow,
~1-3 ms for a CUB-sized photo), converts and normalises it -- at the HIP forward's
~2,800 images/s that host work is the bottleneck.

MI355X split:
  * host workers only decode (``Image.open(f).convert('RGB')``, torchvision's
    ``pil_loader``); a batch is packed into ONE pinned uint8 buffer (ragged HWC images +
    offsets + sizes) -- one H2D copy per batch of ~0.5 MB/image instead of 0.6 MB of fp32;
  * the device does Resize + [Grayscale(3)] + ToTensor + Normalize in one launch
    (``pipnet_resize_normalize_rgb8``), bit-identical to Pillow + torchvision
    (oracle/input_ref.py), writing the NCHW fp32 batch the backbone reads.

``ImageFolder`` semantics (class discovery, sample order, extensions, errors) follow
torchvision.datasets.folder (third party, absent here) so ``classes`` / ``targets`` and the
order of evaluation match the reference's loaders exactly.
"""
from __future__ import annotations

import os
from typing import Callable, Dict, List, NamedTuple, Optional, Sequence, Tuple

import numpy as np
import torch

IMG_EXTENSIONS = (".jpg", ".jpeg", ".png", ".ppm", ".bmp", ".pgm", ".tif", ".tiff", ".webp")
IMAGENET_MEAN = (0.485, 0.456, 0.406)      # util/data.py:262-263 (and every get_* of it)
IMAGENET_STD = (0.229, 0.224, 0.225)


# ---- torchvision.datasets.folder semantics ------------------------------------------------

def find_classes(directory: str) -> Tuple[List[str], Dict[str, int]]:
    """Class folders sorted by name -> index (torchvision ``find_classes``)."""
    classes = sorted(entry.name for entry in os.scandir(directory) if entry.is_dir())
    if not classes:
        raise FileNotFoundError(f"Couldn't find any class folder in {directory}.")
    return classes, {c: i for i, c in enumerate(classes)}


def has_file_allowed_extension(filename: str, extensions: Sequence[str]) -> bool:
    return filename.lower().endswith(tuple(extensions))


def make_dataset(directory: str, class_to_idx: Dict[str, int],
                 extensions: Sequence[str] = IMG_EXTENSIONS) -> List[Tuple[str, int]]:
    """(path, class index) for every allowed file, classes in sorted order, each class's
    tree walked in sorted order (torchvision ``make_dataset``)."""
    directory = os.path.expanduser(directory)
    instances, available = [], set()
    for target_class in sorted(class_to_idx.keys()):
        class_index = class_to_idx[target_class]
        target_dir = os.path.join(directory, target_class)
        if not os.path.isdir(target_dir):
            continue
        for root, _, fnames in sorted(os.walk(target_dir, followlinks=True)):
            for fname in sorted(fnames):
                path = os.path.join(root, fname)
                if has_file_allowed_extension(path, extensions):
                    instances.append((path, class_index))
                    available.add(target_class)
    empty = set(class_to_idx.keys()) - available
    if empty:
        raise FileNotFoundError(f"Found no valid file for the classes {', '.join(sorted(empty))}. "
                                f"Supported extensions are: {', '.join(extensions)}")
    return instances


def decode_rgb(path: str) -> np.ndarray:
    """torchvision ``pil_loader``: ``Image.open(f).convert('RGB')`` -> HxWx3 uint8."""
    from PIL import Image
    with open(path, "rb") as f:
        img = Image.open(f)
        return np.asarray(img.convert("RGB"), dtype=np.uint8)


class DecodedImageFolder(torch.utils.data.Dataset):
    """ImageFolder that stops after decoding: ``ds[i] -> (HxWx3 uint8 array, target)``.

    Same ``root`` / ``classes`` / ``class_to_idx`` / ``samples`` / ``targets`` / ``imgs`` as
    ``torchvision.datasets.ImageFolder``; the transform runs on the GPU
    (``DeviceEvalTransform``) after ``collate_decoded``."""

    def __init__(self, root: str, loader: Callable[[str], np.ndarray] = decode_rgb,
                 extensions: Sequence[str] = IMG_EXTENSIONS):
        self.root = os.fspath(root)
        self.classes, self.class_to_idx = find_classes(self.root)
        self.samples = make_dataset(self.root, self.class_to_idx, extensions)
        self.targets = [s[1] for s in self.samples]
        self.imgs = self.samples
        self.loader = loader

    def __len__(self) -> int:
        return len(self.samples)

    def __getitem__(self, index: int):
        path, target = self.samples[index]
        return self.loader(path), target


class PackedImages(NamedTuple):
    """A ragged batch of decoded images in one buffer (host, pinnable, or device)."""
    pixels: torch.Tensor     # [sum(h*w*3)] uint8, image b at pixels[offsets[b]:]
    offsets: torch.Tensor    # [B] int64
    sizes: torch.Tensor      # [B, 2] int32 (h, w)
    targets: torch.Tensor    # [B] int64


def pack_images(images: Sequence[np.ndarray], targets: Optional[Sequence[int]] = None) -> PackedImages:
    """Pack HxWx3 uint8 images into one contiguous buffer (the DataLoader collate)."""
    b = len(images)
    sizes = np.zeros((b, 2), np.int32)
    offsets = np.zeros(b, np.int64)
    total = 0
    for i, im in enumerate(images):
        if im.dtype != np.uint8 or im.ndim != 3 or im.shape[2] != 3:
            raise ValueError(f"image {i}: expected HxWx3 uint8 RGB, got {im.dtype} {im.shape}")
        sizes[i] = im.shape[:2]
        offsets[i] = total
        total += im.size
    pixels = torch.empty(max(total, 1), dtype=torch.uint8)
    flat = pixels.numpy()
    for i, im in enumerate(images):
        flat[offsets[i]:offsets[i] + im.size] = np.ascontiguousarray(im).reshape(-1)
    t = torch.as_tensor(np.asarray(targets if targets is not None else [-1] * b, dtype=np.int64))
    return PackedImages(pixels, torch.from_numpy(offsets), torch.from_numpy(sizes), t)


def collate_decoded(batch) -> PackedImages:
    """``DataLoader(collate_fn=...)`` for ``DecodedImageFolder`` items."""
    return pack_images([im for im, _ in batch], [t for _, t in batch])


class DeviceEvalTransform:
    """``transform_no_augment`` on the GPU: Resize(size) [+ Grayscale(3)] + ToTensor +
    Normalize(mean, std) of a ``PackedImages`` batch -> [B,3,h,w] fp32 on ``device``.
    Bit-identical to the reference's Pillow / torchvision transform (oracle/input_ref.py)."""

    def __init__(self, size, mean=IMAGENET_MEAN, std=IMAGENET_STD, grayscale: bool = False):
        self.size = (int(size), int(size)) if isinstance(size, int) else (int(size[0]), int(size[1]))
        self.mean = tuple(float(v) for v in mean)
        self.std = tuple(float(v) for v in std)
        self.grayscale = bool(grayscale)

    def __call__(self, packed: PackedImages, device, want_u8: bool = False):
        from . import kernels as K
        dev = torch.device(device)
        if dev.type != "cuda":
            raise RuntimeError("DeviceEvalTransform runs on a ROCm device only (there is no CPU fallback)")
        sizes_host = packed.sizes.cpu().numpy() if packed.sizes.is_cuda else packed.sizes.numpy()
        pixels = packed.pixels.to(dev, non_blocking=True)
        offsets = packed.offsets.to(dev, non_blocking=True)
        sizes = packed.sizes.to(dev, non_blocking=True)
        return K.resize_normalize_rgb8(pixels, offsets, sizes, sizes_host, self.size, self.mean, self.std,
                                       self.grayscale, want_u8)


class DeviceEvalLoader:
    """Iterates ``(xs, ys)`` device batches like the reference's test loader followed by
    ``xs.to(device), ys.to(device)`` (pipnet/test.py:67-69): host workers decode and pack,
    the device transforms.  ``len()`` and ``dataset`` as a DataLoader's."""

    def __init__(self, dataset: DecodedImageFolder, transform: DeviceEvalTransform, device, batch_size: int,
                 num_workers: int = 0, shuffle: bool = False, drop_last: bool = False):
        self.dataset = dataset
        self.transform = transform
        self.device = torch.device(device)
        self.loader = torch.utils.data.DataLoader(dataset, batch_size=batch_size, shuffle=shuffle,
                                                  num_workers=num_workers, collate_fn=collate_decoded,
                                                  pin_memory=True, drop_last=drop_last)
        self.batch_size = batch_size

    def __len__(self) -> int:
        return len(self.loader)

    def __iter__(self):
        for packed in self.loader:
            xs = self.transform(packed, self.device)
            yield xs, packed.targets.to(self.device, non_blocking=True)


def get_eval_loader(test_dir: str, img_size: int, batch_size: int, device, num_workers: int = 8,
                    grayscale: bool = False, mean=IMAGENET_MEAN, std=IMAGENET_STD,
                    shuffle: bool = True) -> DeviceEvalLoader:
    """The reference's ``testloader`` (util/data.py:199-206: ``ImageFolder(test_dir,
    transform_no_augment)``, ``batch_size=args.batch_size``, ``shuffle=True``,
    ``drop_last=False``) with the transform on the GPU.  eval_pipnet's metrics do not
    depend on the order; ``shuffle=False`` gives the projection loaders' order."""
    ds = DecodedImageFolder(test_dir)
    return DeviceEvalLoader(ds, DeviceEvalTransform(img_size, mean, std, grayscale), device, batch_size,
                            num_workers=num_workers, shuffle=shuffle)
