"""Summarise scripts/pmc_var_traffic.sh passes into per-launch HBM traffic of the variable-length
encode / decode pipelines (C3 mixed, C4 nested bench workloads).

Per kernel: median FETCH_SIZE / WRITE_SIZE (KB per dispatch) over the bench's dispatches, with the
gfx950 corrections of MI355X_MICROARCH.md §HBM as calibrated on tools/hbm_probe in
profiles/pmc_struct100.json (FETCH_SIZE counts half of the bytes of 8- and 16-B-per-lane reads:
x2; WRITE_SIZE exact: x1).  Encode = measure_tiles + encode_var_reg + the scan kernels (the bench's untimed
pre-size, measure_kernel + add_group_prefix, is listed but not counted);
decode = decode_var_reg (decode_measure_* run only in the untimed sizing path).  Algorithmic bytes per launch come from the bench line in the same
pass's log (encode and decode both move column bytes + row bytes: half of a step).

usage: python3 scripts/pmc_var_summarize.py <pmc dir> <workload>
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


def bench_line(log):
    for line in open(log):
        line = line.strip()
        if line.startswith("{") and '"metric"' in line:
            return json.loads(line)
    raise SystemExit(f"no bench line in {log}")


def short(name):
    return name.replace("fury::(anonymous namespace)::", "").replace("void ", "").split("(")[0]


def main():
    root, w = sys.argv[1], sys.argv[2]
    fetch = load(os.path.join(root, f"{w}_FETCH_SIZE"), "FETCH_SIZE")
    write = load(os.path.join(root, f"{w}_WRITE_SIZE"), "WRITE_SIZE")
    bl = bench_line(os.path.join(root, f"{w}_FETCH_SIZE.log"))
    alg = bl["config"]["algorithmic_bytes_per_step_per_gpu"] / 2
    kernels = {}
    for k in sorted(set(fetch) | set(write)):
        if "fury::" not in k:
            continue
        fb = fetch.get(k, 0.0) * 1024 * FETCH_FACTOR
        wb = write.get(k, 0.0) * 1024 * WRITE_FACTOR
        kernels[short(k)] = {"kernel": k, "FETCH_SIZE_KB": fetch.get(k), "WRITE_SIZE_KB": write.get(k),
                             "fetch_bytes_corrected": round(fb), "write_bytes_corrected": round(wb),
                             "hbm_bytes_per_launch": round(fb + wb)}
    # the timed encode is fury_row_encode_measured: measure_tiles + scans + encode_var_reg; the
    # row-sized measure_kernel + add_group_prefix only pre-size the bench's buffer (untimed)
    timed = ("encode_var", "measure_tiles", "scan_", "add_groups") if any(
        n.startswith("measure_tiles") for n in kernels) else (
        "encode_var", "measure_kernel", "add_group_prefix", "scan_", "add_groups")
    enc = sum(v["hbm_bytes_per_launch"] for n, v in kernels.items() if n.startswith(timed))
    dec = sum(v["hbm_bytes_per_launch"] for n, v in kernels.items()
              if n.startswith("decode_var"))
    res = {"method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over "
                     f"`bench.py --workload {w} --steps 3 --warmup 1`; KB per dispatch (median); "
                     "FETCH x2 / WRITE x1 (gfx950 corrections, calibrated in pmc_struct100.json)",
           "workload": w, "rows": bl["config"]["rows_per_gpu"],
           "algorithmic_bytes_per_launch": alg,
           "encode_hbm_bytes_per_launch": enc, "decode_hbm_bytes_per_launch": dec,
           "encode_traffic_over_algorithmic": round(enc / alg, 4),
           "decode_traffic_over_algorithmic": round(dec / alg, 4),
           "kernels": kernels}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
