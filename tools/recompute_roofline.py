"""Recompute every roofline `frac` of a bench line from a rocprofv3 kernel-stats CSV of the same
tree: frac = algorithmic GFLOP per launch / average launch duration / peak,
with the GFLOP per launch from DESIGN.md's formulas (bench.py writes them into each roofline
block) and the duration from the CSV's AverageNs for the same kernel name.

    python tools/recompute_roofline.py [profiles/r04/bench_final.json] [profiles/r04/kernel_stats_bench_final.csv]
"""
import csv
import json
import sys


def blocks(line):
    yield "headline (C2)", line["roofline"]
    for name, ex in line.get("extra", {}).items():
        yield f"extra.{name}", ex["roofline"]
    if "roofline" in line.get("alt_precision", {}):
        yield "alt_precision", line["alt_precision"]["roofline"]


def main():
    bench = sys.argv[1] if len(sys.argv) > 1 else "profiles/r04/bench_final.json"
    stats = sys.argv[2] if len(sys.argv) > 2 else "profiles/r04/kernel_stats_bench_final.csv"
    line = json.loads(open(bench).read().strip().splitlines()[-1])
    avg = {}
    for row in csv.DictReader(open(stats)):
        name = row["Name"]
        key = name.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").strip()
        avg[key] = (float(row["AverageNs"]) / 1e3, int(row["Calls"]))
    print(f"{'block':15s} {'kernel':62s} {'GFLOP':>8s} {'bench us':>9s} {'csv us':>8s} {'calls':>6s} "
          f"{'frac(bench)':>11s} {'frac(csv)':>9s}")
    for tag, rf in blocks(line):
        k = rf["kernel"]
        us, calls = avg.get(k, (float("nan"), 0))
        g = rf["algorithmic_gflop_per_launch"]
        frac_csv = g / (us * 1e-6) / (rf["peak"] * 1e3) if calls else float("nan")
        print(f"{tag:15s} {k[:62]:62s} {g:8.2f} {rf['avg_launch_us']:9.1f} {us:8.1f} {calls:6d} "
              f"{rf['frac']:11.4f} {frac_csv:9.4f}")


if __name__ == "__main__":
    main()
