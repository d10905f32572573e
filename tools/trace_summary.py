"""Summarise a rocprofv3 kernel_trace.csv: per-kernel count / total / avg / share."""
import csv
import sys
from collections import defaultdict

agg = defaultdict(lambda: [0, 0.0])
with open(sys.argv[1]) as f:
    for row in csv.DictReader(f):
        d = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-3  # us
        a = agg[row["Kernel_Name"][:90]]
        a[0] += 1
        a[1] += d
tot = sum(v[1] for v in agg.values())
print(f"{'kernel':90s} {'calls':>8s} {'total_ms':>10s} {'avg_us':>9s} {'share':>6s}")
for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:40]:
    print(f"{k:90s} {n:8d} {t/1e3:10.1f} {t/n:9.2f} {100*t/tot:5.1f}%")
print(f"total kernel time {tot/1e3:.1f} ms over {sum(v[0] for v in agg.values())} dispatches")
