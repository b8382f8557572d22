"""TEST-ONLY stand-in for the third-party ``torchvision`` package.

torchvision is not installed in this image.  The
reference's ``features/convnext_features.py:3,50-51,79-80`` imports
``torchvision.models.convnext_tiny`` / ``ConvNeXt_Tiny_Weights``.  This
package restates exactly that surface (ConvNeXt-tiny)
so that ``tests/golden/gen_golden.py`` can import the reference's own
``pipnet/*.py`` and ``features/*.py`` unchanged and record golden vectors.

It is used by nothing else: not by the product package, not on the GPU box.
"""
from . import models  # noqa: F401
