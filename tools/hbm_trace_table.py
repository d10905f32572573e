"""Per-configuration kernel time from a rocprofv3 kernel trace of tools/bench_hbm_kernels.py.

Dispatches are ordered by start time and split at the marker launches (dd_synth_images_u8,
one just before and one just after each configuration's timed calls); the configuration's time per call =
the summed duration of every dispatch in its segment (all kernels of a select_topk call)
divided by its call count.  Prints a table and writes JSON (argv[3]) with achieved GB/s and
the fraction of 8 TB/s next to the HIP-event figure of the same run.

    python tools/hbm_trace_table.py kernel_trace.csv sweep.json [out.json]
"""
import csv
import json
import sys


def main():
    trace, sweep = sys.argv[1], sys.argv[2]
    with open(sweep) as f:
        cfgs = json.load(f)
    rows = []
    with open(trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    segs, cur = [], None
    for s, e, name in rows:
        if "synth" in name:
            cur = []
            segs.append(cur)
        elif cur is not None:
            cur.append((s, e, name))
    # markers bracket each configuration's timed calls: segments alternate
    # [timed calls of config i] [warm-up of config i+1] ... [nothing after the last marker]
    segs = segs[0::2]
    if len(segs) < len(cfgs):
        raise SystemExit(f"{len(segs)} marked segments vs {len(cfgs)} configurations")
    out = []
    print(f"{'kernel':12s} {'shape':28s} {'bytes/call':>12s} {'trace_us':>10s} {'event_us':>10s}"
          f" {'GB/s':>8s} {'frac':>6s}  kernels/call")
    for c, seg in zip(cfgs, segs):
        per_call = len(seg) / c["iters"]
        t_us = sum((e - s) * 1e-3 for s, e, _ in seg) / c["iters"]
        gbps = c["bytes"] / (t_us * 1e-6) / 1e9
        shape = ", ".join(f"{k}={c[k]}" for k in ("C", "rows", "images", "n", "k", "dist") if k in c)
        print(f"{c['kernel']:12s} {shape:28s} {c['bytes']:12d} {t_us:10.1f} {c['us']:10.1f} "
              f"{gbps:8.0f} {gbps / 8000:6.3f}  {per_call:g}")
        if per_call > 1 and per_call == int(per_call):
            # one call's dispatches in launch order (the last timed call)
            one = seg[-int(per_call):]
            short = lambda nm: nm.split("(")[0].split("::")[-1].replace("void ", "")  # noqa: E731
            print("    " + " ".join(f"{short(nm)}:{(e - s) * 1e-3:.1f}" for s, e, nm in one))
        out.append(dict(c, trace_us=t_us, trace_GBps=gbps, trace_frac=gbps / 8000.0,
                        kernels_per_call=per_call))
    if len(sys.argv) > 3:
        with open(sys.argv[3], "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
