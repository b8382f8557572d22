"""Interleaved A/B of a switch of the HIP path on one BASELINE config, in one process
(cdna_hip_programming.md rule 24): rounds of per-arm timings of net(xs, inference=True).

    python tools/ab_toggle.py <module>.<FLAG> <config> [--rounds 5] [--steps 10]
e.g. count_pipnet_amd.resnet_hip.DUAL_1X1 c3  (arms False, True)
Stream splits as arms: streams:1:2:3.
An int module attribute per arm: attr:<module>.<NAME>:<v>:<v>[...].
A library switch function instead of a module flag: fn:<module>.<func>:<arg>:<arg>[:<arg>...],
one arm per argument, e.g. fn:module.setter:0:1 (a setter function called with each value).  Prints one JSON line per arm and whether
every arm's outputs are bitwise equal to the first arm's."""
import argparse
import importlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import bench_configs as bc  # noqa: E402
from count_pipnet_amd.synthetic import synth_images  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("flag")
    ap.add_argument("config")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--stream-split", type=int, default=0, help="0 = the model's default")
    a = ap.parse_args()
    net_holder = {}
    if a.flag.startswith("streams:"):            # arms = stream splits of the model itself
        arms = [int(v) for v in a.flag.split(":")[1:]]

        def switch(val):
            from count_pipnet_amd.pipnet import set_stream_split
            set_stream_split(net_holder["net"], val)
    elif a.flag.startswith("fn:"):
        parts = a.flag.split(":")
        modname, fname = parts[1].rsplit(".", 1)
        fn = getattr(importlib.import_module(modname), fname)
        arms = [int(v) for v in parts[2:]]

        def switch(val):
            fn(val)
    elif a.flag.startswith("attr:"):           # attr:<module>.<NAME>:<v>:<v>... -- an int module attribute per arm
        parts = a.flag.split(":")
        modname, attr = parts[1].rsplit(".", 1)
        mod = importlib.import_module(modname)
        arms = [int(v) for v in parts[2:]]

        def switch(val):
            setattr(mod, attr, val)
    else:
        modname, attr = a.flag.rsplit(".", 1)
        mod = importlib.import_module(modname)
        arms = [False, True]

        def switch(val):
            setattr(mod, attr, val)
    dev = torch.device("cuda:0")
    cfg = bc.CONFIGS[a.config]
    net = bc.make(cfg, dev)
    net_holder["net"] = net
    xs = synth_images(cfg["batch"], cfg["size"], seed=1).to(dev)
    if a.stream_split:
        from count_pipnet_amd.pipnet import set_stream_split
        set_stream_split(net, a.stream_split)
    res = {v: [] for v in arms}
    outs = {}
    with torch.no_grad():
        for r in range(a.rounds):
            for val in arms:
                switch(val)
                for _ in range(2):
                    o = net(xs, inference=True)
                torch.cuda.synchronize()
                if r == 0:
                    outs[val] = [t.float().clone() for t in o]
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.steps):
                    net(xs, inference=True)
                e1.record()
                torch.cuda.synchronize()
                res[val].append(e0.elapsed_time(e1) / a.steps)
    switch(arms[0])
    for val in arms:
        ms = sorted(res[val])
        print(json.dumps({"flag": a.flag, "value": val, "config": a.config, "stream_split": a.stream_split or "default",
                          "ms_median": ms[len(ms) // 2], "ms_min": ms[0],
                          "img_s_median": cfg["batch"] / ms[len(ms) // 2] * 1e3,
                          "bitwise_equal_to_first_arm": all(torch.equal(x, y) for x, y in
                                                            zip(outs[arms[0]], outs[val]))}))


if __name__ == "__main__":
    main()
