"""Summarise scripts/r04_nested_prof.sh (4M depth-3 nested rows through the default engines:
row-walk measure + encode, row-walk decode) into per-dispatch HBM traffic per kernel.

Median FETCH_SIZE / WRITE_SIZE (KB per dispatch) with the gfx950 corrections calibrated in
profiles/pmc_struct100.json (FETCH x2, WRITE x1), over the batch's row bytes (1.20 GB) and column
bytes (0.40 GB) printed by scripts/ab_generic.py.

usage: python3 scripts/pmc_generic_summarize.py <r04n dir>
"""
import csv
import glob
import json
import os
import statistics
import sys

FETCH_FACTOR = 2.0
WRITE_FACTOR = 1.0


def load(dirpath, counter):
    out = {}
    for f in glob.glob(os.path.join(dirpath, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if r.get("Counter_Name") == counter:
                    out.setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]))
    return {k: statistics.median(v) for k, v in out.items()}


def sizes(log):
    for line in open(log):
        if line.startswith("{") and "row_bytes" in line:
            d = json.loads(line)
            return d["row_bytes"], d["column_bytes"]
    raise SystemExit(f"no size line in {log}")


def short(name):
    return name.replace("fury::(anonymous namespace)::", "").replace("void ", "").split("(")[0]


def main():
    root = sys.argv[1]
    fetch = load(os.path.join(root, "FETCH_SIZE"), "FETCH_SIZE")
    write = load(os.path.join(root, "WRITE_SIZE"), "WRITE_SIZE")
    rb, cb = sizes(os.path.join(root, "FETCH_SIZE.log"))
    kernels = {}
    for k in sorted(set(fetch) | set(write)):
        if "fury::" not in k:
            continue
        fb = fetch.get(k, 0.0) * 1024 * FETCH_FACTOR
        wb = write.get(k, 0.0) * 1024 * WRITE_FACTOR
        kernels[short(k)] = {"fetch_bytes": round(fb), "write_bytes": round(wb),
                             "fetch_over_row_bytes": round(fb / rb, 3),
                             "write_over_row_bytes": round(wb / rb, 3)}
    print(json.dumps({"method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes over "
                                "scripts/ab_generic.py --rows 4000000 --iters 1 (default engines: "
                                "row-walk measure + encode, row-walk decode); KB per dispatch "
                                "(median); corrected FETCH x2 / WRITE x1 (gfx950, "
                                "profiles/pmc_struct100.json calibration)",
                      "rows": 4000000, "row_bytes": rb, "column_bytes": cb, "kernels": kernels},
                     indent=1))


if __name__ == "__main__":
    main()
