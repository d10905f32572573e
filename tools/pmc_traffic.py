"""Per-kernel-kind HBM bytes per dispatch from tools/pmc_bench.sh's FETCH_SIZE / WRITE_SIZE
passes, keyed like bench.py's kernel kinds (profiles/pmc_traffic.json).

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports half the bytes of a wide
coalesced streaming read (16 B/lane loads: our staging and weight loads), so reads are
counted x2; WRITE_SIZE is exact for 16-B/lane stores and reported as is (our epilogue stores
are 4 B/lane, 128-B segments: uncalibrated, so the raw value is kept alongside).  Both
counters tally fabric-side requests, i.e. Infinity-Cache hits are included."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

KIND = {"conv3x3_kernel": "conv3x3", "conv3x3_r2_kernel": "conv3x3",
        "pegrad_direct3x3_kernel": "direct3x3", "pegrad_direct3x3p_kernel": "direct3x3",
        "down_fwd_kernel": "down_fwd",
        "down_bwd_kernel": "down_bwd", "down_bwd2_kernel": "down_bwd", "apply_kernel": "bn_apply",
        "pgram_kernel": "pgram"}



def _staging_mode(kernel_name):
    """The XF template argument (6th) of a conv3x3 / conv3x3_r2 kernel name, 0 if absent."""
    if "<" not in kernel_name:
        return 0
    args = kernel_name.split("<", 1)[1].split(">", 1)[0].split(",")
    try:
        return int(args[5].strip())
    except (IndexError, ValueError):
        return 0  # (a bool XF: the builds before the fused unit input)


vals = defaultdict(lambda: defaultdict(list))
for counter in ("FETCH_SIZE", "WRITE_SIZE"):
    for fn in glob.glob(os.path.join(sys.argv[1], counter, "**", "*counter_collection.csv"),
                        recursive=True):
        with open(fn) as f:
            for row in csv.DictReader(f):
                if row.get("Counter_Name") != counter:
                    continue
                kn = row["Kernel_Name"]
                for k, kind in KIND.items():
                    if k in kn:
                        if kind == "conv3x3" and _staging_mode(kn) >= 2:
                            kind = "conv3x3_unit"  # the fused residual-unit input (kXfOut*)
                        vals[kind][counter].append(float(row["Counter_Value"]) * 1024.0)
                        break
out = {}
for kind, d in vals.items():
    f, w = d.get("FETCH_SIZE"), d.get("WRITE_SIZE")
    if not f or not w:
        continue
    fa, wa = sum(f) / len(f), sum(w) / len(w)
    out[kind] = {"hbm_bytes_per_launch": 2 * fa + wa, "fetch_bytes_raw": fa, "write_bytes": wa,
                 "dispatches": len(f),
                 "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes) over "
                           "bench.py --n 10240 --ckpts 1 --steps 1; FETCH x2 (gfx950 "
                           "streaming-read correction); per-dispatch mean over all shapes"}
print(json.dumps(out, indent=1))
