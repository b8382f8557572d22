"""count_pipnet_amd -- MI355X-native PIP-Net / CountPIPNet inference path.

Drop-in for the reference's ``pipnet.pipnet`` / ``pipnet.count_pipnet`` forward hot path
(backbone -> add-on -> per-patch softmax / Gumbel-argmax -> max-pool / count -> sparse
non-negative linear head), executed by hand-written HIP kernels for gfx950 behind the
C-ABI declared in ``include/pipnet_amd.h``.
"""
__version__ = "0.1.0"

from .backend import invalidate_weight_caches, torch_backend  # noqa: E402,F401
