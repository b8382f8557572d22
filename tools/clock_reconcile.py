"""Reconcile the two clock figures of the fp32 GEMM: the PMC quotient
GRBM_GUI_ACTIVE / 8 / wall and the in-kernel s_memtime / s_memrealtime ratio, taken on the SAME
dispatch.  tools/gemm_stamps.py runs each shape 4x and prints the stamps clock of its last
launch with the grid size; this script finds that dispatch in the rocprofv3 counter CSV (same
Grid_Size, highest Dispatch_Id) and prints, per shape:
  wall (kernel trace), clk_stamps, clk_grbm = GRBM_GUI_ACTIVE / 8 / wall,
  clk_sq = SQ_BUSY_CYCLES / 32 / wall (32 shader engines), and the MFMA busy fraction at each
  clock (SQ_VALU_MFMA_BUSY_CYCLES = 64 cycles per 32x32x2 f32 MFMA, summed over 1,024 SIMDs).
    python tools/clock_reconcile.py <rocprof dir> <stamps log>
"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def main():
    pdir, log = sys.argv[1], sys.argv[2]
    rows = []
    for f in glob.glob(os.path.join(pdir, "**", "*counter_collection.csv"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    disp = defaultdict(dict)
    for r in rows:
        d = disp[int(r["Dispatch_Id"])]
        d["grid"] = int(r["Grid_Size"])
        d[r["Counter_Name"]] = float(r["Counter_Value"])
        if "Start_Timestamp" in r:
            d["wall_ns"] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    last = {}
    for i in sorted(disp):
        last[disp[i]["grid"]] = disp[i]
    print(f"{'shape':10s} {'grid':>9s} {'wall_us':>9s} {'clk_stamp':>9s} {'clk_grbm':>9s} {'clk_sq':>7s} "
          f"{'busy@grbm':>9s} {'busy@stamp':>10s} {'TF/s':>7s} {'frac_spec':>9s}")
    for line in open(log):
        m = re.match(r"(\S+)\s+v\d+ M=(\d+) N=(\d+) K=(\d+) wg=\d+ grid=(\d+) .*clk=([\d.]+)GHz", line)
        if not m:
            continue
        name, mm, nn, kk, grid, clk = m.group(1), *map(int, m.group(2, 3, 4, 5)), float(m.group(6))
        d = last.get(grid)
        if d is None or "wall_ns" not in d:
            print(f"{name:10s} {grid:9d}  (no counter row)")
            continue
        w = d["wall_ns"] * 1e-9
        g = d.get("GRBM_GUI_ACTIVE", 0) / 8 / w / 1e9
        sq = d.get("SQ_BUSY_CYCLES", 0) / 32 / w / 1e9
        mf = d.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / 1024            # per-SIMD busy cycles
        tf = 2.0 * mm * nn * kk / w / 1e12
        print(f"{name:10s} {grid:9d} {w * 1e6:9.1f} {clk:9.2f} {g:9.2f} {sq:7.2f} {mf / (g * 1e9 * w):9.3f} "
              f"{mf / (clk * 1e9 * w):10.3f} {tf:7.1f} {tf / 157.3:9.3f}")


if __name__ == "__main__":
    main()
