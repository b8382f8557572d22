"""Per-kernel mean of every PMC counter found under a tools/pmc_generic.sh output dir, plus the
mean kernel duration (us) of each pass."""
import csv
import glob
import os
import re
import sys
from collections import defaultdict

d = sys.argv[1]
agg = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        m = re.search(r"((?:\w+::)*\w+)(<[^(]*>)?\(", r.get("Kernel_Name", ""))
        k = (m.group(1) + (m.group(2) or "")) if m else r.get("Kernel_Name", "")[:80]
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        if "Start_Timestamp" in r:
            agg[k]["dur_us"].append((float(r["End_Timestamp"]) - float(r["Start_Timestamp"])) / 1e3)
for k, c in agg.items():
    print(k[:150])
    for name, v in sorted(c.items()):
        print(f"    {name:32s} n={len(v):4d} mean={sum(v) / len(v):.6g}")
