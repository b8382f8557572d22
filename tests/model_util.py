"""Build the product's models for a golden case (same factories as main.py:105-115)."""
import contextlib
import io

import torch

from count_pipnet_amd.count_pipnet import get_count_network
from count_pipnet_amd.pipnet import get_pipnet
from count_pipnet_amd.synthetic import fill_module_
from golden_util import golden_args


def build_model(meta):
    case = meta["case"]
    args = golden_args(meta)
    with contextlib.redirect_stdout(io.StringIO()):
        if case["model"] == "pipnet":
            net, _ = get_pipnet(case["num_classes"], args)
        else:
            net, _ = get_count_network(case["num_classes"], args, max_count=case["max_count"], use_ste=case["use_ste"])
    fill_module_(net, case["seed"], meta["profile"])
    return net.eval()
