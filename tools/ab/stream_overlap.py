"""Experiment: C2 forward as two concurrent half-batch forwards on two HIP streams (dwconv /
LayerNorm / head kernels of one half co-resident with the MFMA GEMMs of the other) vs one
full-batch forward.  python tools/stream_overlap.py"""
import argparse
import contextlib
import io
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from count_pipnet_amd import build  # noqa: E402
from count_pipnet_amd.pipnet import get_pipnet  # noqa: E402
from count_pipnet_amd.synthetic import fill_module_, synth_images  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--splits", default="1,2,4")
    a = ap.parse_args()
    build.build()
    dev = torch.device("cuda:0")
    args = argparse.Namespace(net="convnext_tiny_26", disable_pretrained=True, num_features=0, bias=False)
    with contextlib.redirect_stdout(io.StringIO()):
        net, _ = get_pipnet(200, args)
    fill_module_(net, 7, "trained")
    net = net.eval().to(dev)
    xs = synth_images(64, 224, seed=5).to(dev)
    res = {}
    with torch.no_grad():
        ref = net(xs, inference=True)
        for ns in [int(v) for v in a.splits.split(",")]:
            streams = [torch.cuda.Stream(device=dev) for _ in range(ns)]
            parts = xs.chunk(ns)

            def step():
                main = torch.cuda.current_stream(dev)
                outs = []
                for s, p in zip(streams, parts):
                    s.wait_stream(main)
                    with torch.cuda.stream(s):
                        outs.append(net(p, inference=True))
                for s in streams:
                    main.wait_stream(s)
                return outs
            for _ in range(3):
                outs = step()
            torch.cuda.synchronize()
            ok = all(torch.equal(torch.cat([o[i] for o in outs]), ref[i]) for i in (1, 2))
            t0 = time.perf_counter()
            for _ in range(a.steps):
                step()
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / a.steps * 1e3
            res[f"streams{ns}"] = dict(ms_per_step=ms, images_per_sec=64 / ms * 1e3, identical_to_full_batch=ok)
            print(json.dumps({f"streams{ns}": res[f"streams{ns}"]}), flush=True)


if __name__ == "__main__":
    main()
