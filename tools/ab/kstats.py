"""Print the top kernels of a rocprofv3 --stats kernel summary: share of kernel time, calls,
average us, name.   python tools/kstats.py <run_kernel_stats.csv> [top] [calls_per_step]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
per = float(sys.argv[3]) if len(sys.argv) > 3 else 0.0
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in rows[:top]:
    t, n, avg = float(r["TotalDurationNs"]), int(r["Calls"]), float(r["AverageNs"]) / 1e3
    step = f" {t / per / 1e3:8.1f}us/step" if per else ""
    print(f"{t / tot * 100:5.1f}% {n:6d} {avg:9.1f}us{step}  {r['Name'][:110]}")
print(f"total {tot / 1e6:.3f} ms")
