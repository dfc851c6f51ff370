"""Summarise rocprofv3 FETCH_SIZE / WRITE_SIZE passes (scripts/pmc.sh) into per-launch HBM
traffic for the Struct-100 encode/decode kernels.

Corrections follow MI355X_MICROARCH.md §HBM: FETCH_SIZE under-reports wide coalesced reads by 2x
on gfx950 and WRITE_SIZE is exact for 16-B-per-lane streaming stores; other widths are
calibrated here on tools/hbm_probe kernels that move a known number of bytes with the same
access width (read_k: 16 B/lane, read8_k / write8_k: 8 B/lane, write_k: 16 B/lane).
"""
import csv
import glob
import json
import os
import statistics
import sys

PROBE_BYTES = 855638016


def load(dirpath):
    rows = []
    for f in glob.glob(os.path.join(dirpath, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            rows.extend(csv.DictReader(fh))
    return rows


def per_kernel(rows, counter):
    out = {}
    for r in rows:
        if r.get("Counter_Name") != counter:
            continue
        out.setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]))
    return out


def pick(d, *needles):
    for k, v in d.items():
        if all(n in k for n in needles):
            return statistics.median(v), k
    return None, None


def main():
    root = sys.argv[1]
    res = {"method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; "
                     "values in KB per dispatch (median over dispatches); calibrated against "
                     "tools/hbm_probe known-byte kernels", "probe_bytes": PROBE_BYTES}
    pf = per_kernel(load(os.path.join(root, "probe_FETCH_SIZE")), "FETCH_SIZE")
    pw = per_kernel(load(os.path.join(root, "probe_WRITE_SIZE")), "WRITE_SIZE")
    bf = per_kernel(load(os.path.join(root, "bench_FETCH_SIZE")), "FETCH_SIZE")
    bw = per_kernel(load(os.path.join(root, "bench_WRITE_SIZE")), "WRITE_SIZE")
    cal = {}
    for name, d, needles in (("fetch16", pf, ("read_k",)), ("fetch8", pf, ("read8_k",)),
                             ("write16", pw, ("write_k",)), ("write8", pw, ("write8_k",))):
        v, k = pick(d, *needles)
        if v:
            cal[name] = {"kernel": k, "counter_KB": v, "factor": PROBE_BYTES / (v * 1024.0)}
    res["calibration"] = cal
    out = {}
    for kind, fneed, wneed, fcal, wcal in (("encode", "encode_fixed", "encode_fixed", "fetch8",
                                            "write16"),
                                           ("decode", "decode_fixed", "decode_fixed", "fetch16",
                                            "write16")):    # pair-mode decode: 16-B stores
        fv, fk = pick(bf, fneed)
        wv, wk = pick(bw, wneed)
        if fv is None or wv is None:
            continue
        ff = cal.get(fcal, {}).get("factor", 2.0)
        wf = cal.get(wcal, {}).get("factor", 1.0)
        fetch_b = fv * 1024 * ff
        write_b = wv * 1024 * wf
        out[kind] = {"kernel": fk, "FETCH_SIZE_KB": fv, "WRITE_SIZE_KB": wv,
                     "fetch_bytes_corrected": fetch_b, "write_bytes_corrected": write_b,
                     "hbm_bytes_per_launch": fetch_b + write_b,
                     "guide_correction_bytes": fv * 1024 * 2 + wv * 1024}
        res[f"{kind}_hbm_bytes_per_launch"] = round(fetch_b + write_b)
    res["kernels"] = out
    alg = {"encode": 1_000_000 * (800 + 816), "decode": 1_000_000 * (816 + 800)}
    res["algorithmic_bytes_per_launch"] = alg
    for k in out:
        res[f"{k}_traffic_over_algorithmic"] = round(out[k]["hbm_bytes_per_launch"] / alg[k], 4)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
