"""Summarise tools/pmc.sh output: per kernel, average duration, effective clock, MFMA busy,
HBM bytes per launch (FETCH_SIZE doubled for the gfx950 wide-read undercount, KB units),
and write profiles/traffic_latest.json for bench.py's roofline.traffic field."""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

d = sys.argv[1]
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from count_pipnet_amd.build import kernel_source_digest  # noqa: E402


def load(pass_dir):
    rows = []
    for f in glob.glob(os.path.join(d, pass_dir, "**", "*counter_collection.csv"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    return rows


def short(name):
    """The kernel's full name with its template arguments (nested ``<...>`` included) and without
    its parameter list -- the key bench.py's launch labels use, so every instantiation gets its own
    row (a regex stopping at the first ``>`` merged e.g. all conv_bf16_kernel<Cfg<...>, ...> tiles)."""
    name = name.replace("(anonymous namespace)::", "").strip()
    if name.startswith("void "):
        name = name[5:]
    depth = 0
    for i, ch in enumerate(name):
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0 and i > 0:
            return name[:i].strip()
    return name.strip()


agg = defaultdict(lambda: defaultdict(list))
for p in ("p1", "p2", "p3"):
    for r in load(p):
        k = short(r.get("Kernel_Name", ""))
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        if "Start_Timestamp" in r and "End_Timestamp" in r and r["Counter_Name"] in ("GRBM_GUI_ACTIVE", "FETCH_SIZE"):
            agg[k]["dur_ns_" + p].append(float(r["End_Timestamp"]) - float(r["Start_Timestamp"]))

out = {}
W = max([48] + [len(k) for k in agg if kernel_source_digest(k) or len(k) <= 64])   # long torch names overflow
print(f"{'kernel':{W}s} {'n':>4s} {'dur_us':>8s} {'clk_GHz':>8s} {'mfma_busy':>9s} {'rd_MB':>9s} {'wr_MB':>9s}")
for k, c in sorted(agg.items(), key=lambda kv: -sum(kv[1].get("dur_ns_p1", [0]))):
    n = len(c.get("GRBM_GUI_ACTIVE", [])) or 1
    dur = sum(c.get("dur_ns_p1", [0])) / max(1, len(c.get("dur_ns_p1", [])))
    grbm = sum(c.get("GRBM_GUI_ACTIVE", [0])) / n
    clk = grbm / 8 / dur if dur else 0.0          # GRBM_GUI_ACTIVE summed over 8 XCDs (cycles)
    busy = sum(c.get("SQ_BUSY_CYCLES", [0])) / n
    mf = sum(c.get("SQ_VALU_MFMA_BUSY_CYCLES", [0])) / n
    nf = len(c.get("FETCH_SIZE", [])) or 1
    nw = len(c.get("WRITE_SIZE", [])) or 1
    rd = 2 * sum(c.get("FETCH_SIZE", [0])) / nf * 1024      # KB -> B, x2 gfx950 wide-read correction
    wr = sum(c.get("WRITE_SIZE", [0])) / nw * 1024
    mfu = mf / (grbm / 8 * 256 * 4) if grbm else 0.0        # per-SIMD busy fraction (cycles units)
    print(f"{k:{W}s} {n:4d} {dur / 1e3:8.1f} {clk:8.2f} {mfu:9.3f} {rd / 1e6:9.1f} {wr / 1e6:9.1f}")
    out[k] = dict(launches=n, avg_us=dur / 1e3, clock_ghz=clk, mfma_busy=mfu, sq_busy=busy,
                  hbm_read_bytes=rd, hbm_write_bytes=wr, hbm_bytes=rd + wr)
json.dump(out, open(os.path.join(d, "summary.json"), "w"), indent=1)
# every kernel whose source family is known -> traffic_kernels.json (bench.py's C3 / C5 roofline
# blocks look their dominant kernel up in profiles/traffic_kernels.json, same digest rule)
METHOD = ("rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes (tools/pmc.sh); "
          "FETCH_SIZE x2 (gfx950 wide-read undercount), KB -> bytes")
per = {k: dict(hbm_bytes_per_launch=v["hbm_bytes"], hbm_read_bytes_per_launch=v["hbm_read_bytes"],
               hbm_write_bytes_per_launch=v["hbm_write_bytes"], avg_us=v["avg_us"], launches=v["launches"],
               mfma_busy=v["mfma_busy"], source_digest=kernel_source_digest(k), method=METHOD)
       for k, v in out.items() if kernel_source_digest(k)}
json.dump(per, open(os.path.join(d, "traffic_kernels.json"), "w"), indent=1)
# the dominant kernel = largest total time (avg x launches) over every MFMA kernel family bench.py
# times (fp32 GEMMs, bf16 convs, fused MLP) -- the same rule as bench.py's roofline block
mfma = {k: v for k, v in out.items() if kernel_source_digest(k)}
if mfma:
    dom = max(mfma, key=lambda k: mfma[k]["avg_us"] * mfma[k]["launches"])
    tr = dict(kernel_key=dom, hbm_bytes_per_launch=mfma[dom]["hbm_bytes"],
              hbm_read_bytes_per_launch=mfma[dom]["hbm_read_bytes"],
              hbm_write_bytes_per_launch=mfma[dom]["hbm_write_bytes"], avg_us=mfma[dom]["avg_us"],
              launches=mfma[dom]["launches"], source_digest=kernel_source_digest(dom),
              method=METHOD)
    if "gemm_f32_tn" in dom:          # the C2 headline's record (bench.py reads traffic_latest first)
        json.dump(tr, open(os.path.join(d, "traffic_latest.json"), "w"), indent=1)
    print("dominant (largest total time):", json.dumps(tr))
