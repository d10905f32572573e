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

# idle gaps on the GPU between consecutive dispatches (same queue order by start time),
# attributed to the kernel that ends each gap: host-side stalls show up here
rows = []
with open(sys.argv[1]) as f:
    for row in csv.DictReader(f):
        rows.append((int(row["Start_Timestamp"]), int(row["End_Timestamp"]),
                     row["Kernel_Name"][:60]))
rows.sort()
gaps = defaultdict(lambda: [0, 0.0])
big = []
idle = 0.0
for (s0, e0, n0), (s1, e1, n1) in zip(rows, rows[1:]):
    g = (s1 - e0) * 1e-3  # us
    if g <= 0:
        continue
    idle += g
    a = gaps[(n0, n1)]
    a[0] += 1
    a[1] += g
    if g > 200:
        big.append((g, n0, n1))
span = (rows[-1][1] - rows[0][0]) * 1e-3 if rows else 0.0
print(f"\nspan {span/1e3:.1f} ms, idle between dispatches {idle/1e3:.1f} ms "
      f"({100 * idle / max(span, 1e-9):.1f}%); {len(big)} gaps > 200 us totalling "
      f"{sum(b[0] for b in big)/1e3:.1f} ms")
print(f"{'after -> before':100s} {'count':>7s} {'idle_ms':>9s}")
for (n0, n1), (c, t) in sorted(gaps.items(), key=lambda kv: -kv[1][1])[:15]:
    print(f"{n0[:48]:48s} -> {n1[:48]:48s} {c:7d} {t/1e3:9.1f}")

# steady state: the timed steps only.  Every bench step ends with one keep-set selection
# (dd_select_topk: hist_top_kernel first, then the split / count / offsets / scatter kernels),
# so the dispatches after the W-th selection (W = warmup steps, argv[2]) are exactly the timed
# steps; their idle share is what a HIP graph could still remove.
SELECT = ("hist_top_kernel", "split_kernel", "count_kernel", "offsets_kernel", "scatter_kernel",
          "clear_kernel", "nan_out_kernel", "lds_order_probe_kernel")
if len(sys.argv) > 2:
    W = int(sys.argv[2])
    starts = [i for i, r in enumerate(rows) if "hist_top_kernel" in r[2]]
    ends = []
    for i in starts:
        j = i
        while j + 1 < len(rows) and any(k in rows[j + 1][2] for k in SELECT):
            j += 1
        ends.append(j)
    if len(ends) > W and W >= 0:
        first = ends[W - 1] + 1 if W > 0 else 0
        tr = rows[first:]
        busy = sum(e - s for s, e, _ in tr) * 1e-3
        gap = sum(max(0, s1 - e0) for (_, e0, _), (s1, _, _) in zip(tr, tr[1:])) * 1e-3
        sp = (tr[-1][1] - tr[0][0]) * 1e-3
        print(f"\ntimed steps (after warmup step {W}): {len(tr)} dispatches, span {sp/1e3:.1f} ms, "
              f"kernel time {busy/1e3:.1f} ms, idle between dispatches {gap/1e3:.1f} ms "
              f"({100 * gap / max(sp, 1e-9):.2f}%)")
