"""Summarise scripts/r05_pmc_walk.sh: per leg, the median WRITE_SIZE and read requests (x 128 B,
every gfx950 fabric read is a 128-B line: profiles/r05_gather_probe.json) of the row-walk and
row-walk-encode kernels, over the 4M-row batch's row bytes / column bytes."""
import csv
import glob
import json
import statistics
import sys

ROWS, COLS = 1202076808, 399060776


def med(d, i, counter, kern):
    vals = []
    for f in glob.glob(f"{d}/{i}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if kern in r["Kernel_Name"] and r["Counter_Name"] == counter:
                vals.append(float(r["Counter_Value"]))
    return statistics.median(vals) if vals else None


d = sys.argv[1]
out = []
for i in range(1, 20):
    try:
        leg = open(f"{d}/leg{i}.txt").read().strip()
    except OSError:
        break
    row = {"leg": leg}
    for k in ("walk_write", "walk_count", "rw_encode", "rw_measure"):
        w = med(d, f"w{i}", "WRITE_SIZE", k)
        r = med(d, f"r{i}", "TCC_EA0_RDREQ_128B_sum", k)
        row[k] = {"write_bytes": None if w is None else int(w * 1024),
                  "write_over_cols": None if w is None else round(w * 1024 / COLS, 3),
                  "read_bytes": None if r is None else int(r * 128),
                  "read_over_rows": None if r is None else round(r * 128 / ROWS, 3)}
    out.append(row)
print(json.dumps(out, indent=1))
