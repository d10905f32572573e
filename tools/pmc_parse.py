"""Per-kernel average FETCH_SIZE / WRITE_SIZE (KB per dispatch) from rocprofv3 --pmc runs.

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE reads 1/2 of the bytes of a wide
coalesced streaming read; our kernels mix 4-B gathers and cached re-reads, for which the
guide has no calibration, so both the raw and the x2-corrected read bytes are reported."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

out = defaultdict(dict)
for counter in ("FETCH_SIZE", "WRITE_SIZE"):
    files = glob.glob(os.path.join(sys.argv[1], counter, "**", "*counter_collection.csv"),
                      recursive=True)
    acc = defaultdict(list)
    for fn in files:
        with open(fn) as f:
            for row in csv.DictReader(f):
                if row.get("Counter_Name") != counter:
                    continue
                acc[row["Kernel_Name"].split("(")[0]].append(float(row["Counter_Value"]))
    for k, v in acc.items():
        out[k][counter + "_KB_avg"] = sum(v) / len(v)
        out[k]["dispatches_" + counter] = len(v)
res = {}
for k, d in out.items():
    f = d.get("FETCH_SIZE_KB_avg")
    w = d.get("WRITE_SIZE_KB_avg")
    if f is not None and w is not None:
        d["hbm_bytes_per_launch_raw"] = (f + w) * 1024
        d["hbm_bytes_per_launch_fetch_x2"] = (2 * f + w) * 1024
    res[k] = d
print(json.dumps(res, indent=1))
