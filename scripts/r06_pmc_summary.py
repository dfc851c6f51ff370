"""Summarise scripts/r06_pmc_walk.sh: per workload and walk kernel, the median WRITE_SIZE (KB
units: x 1024 B) and read requests (x 128 B) per launch, over the batch's row bytes."""
import csv
import glob
import json
import statistics
import sys

ROW_BYTES = {"depth3": 1202076808, "counted128": 2546684000}
COL_BYTES = {"depth3": 399060776}


def med(path, counter, kern):
    vals = []
    for f in glob.glob(f"{path}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if kern in r["Kernel_Name"] and r["Counter_Name"] == counter:
                vals.append(float(r["Counter_Value"]))
    return statistics.median(vals) if vals else None


d = sys.argv[1]
for name, rb in ROW_BYTES.items():
    for kern in ("walk_count", "walk_write"):
        w = med(f"{d}/{name}/w", "WRITE_SIZE", kern)
        rq = med(f"{d}/{name}/r", "TCC_EA0_RDREQ_sum", kern)
        out = {"workload": name, "kernel": kern, "row_bytes": rb,
               "write_bytes": None if w is None else w * 1024,
               "read_bytes": None if rq is None else rq * 128}
        if rq is not None:
            out["read_over_rows"] = round(rq * 128 / rb, 3)
        if w is not None and name in COL_BYTES and kern == "walk_write":
            out["write_over_columns"] = round(w * 1024 / COL_BYTES[name], 3)
        print(json.dumps(out))
