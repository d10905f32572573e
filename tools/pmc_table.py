"""Per-kernel-dispatch-shape average of every PMC counter collected by tools/pmc_conv.sh.
Rows are grouped by (kernel name, grid size) so each microbench shape is one row."""
import csv
import glob
import os
import sys
from collections import defaultdict

acc = defaultdict(lambda: defaultdict(list))
for fn in glob.glob(os.path.join(sys.argv[1], "p*", "**", "*counter_collection.csv"),
                    recursive=True):
    with open(fn) as f:
        for row in csv.DictReader(f):
            name = row["Kernel_Name"].split("(")[0]
            if "pack" in name:
                continue
            key = (name[:60], row.get("Grid_Size", row.get("Grid_Size_X", "?")))
            acc[key][row["Counter_Name"]].append(float(row["Counter_Value"]))
for key in sorted(acc):
    d = acc[key]
    print(f"{key[0]} grid={key[1]}")
    for c in sorted(d):
        v = d[c]
        print(f"    {c:28s} {sum(v) / len(v):16.1f}  (n={len(v)})")
