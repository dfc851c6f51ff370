"""Per-kernel average of every counter in a pmc_var.sh output directory (one line per kernel)."""
import csv, glob, os, sys
from collections import defaultdict

root = sys.argv[1]
for w in sorted({os.path.basename(d).split("_")[0] for d in glob.glob(os.path.join(root, "*_*")) if os.path.isdir(d)}):
    acc = defaultdict(lambda: defaultdict(list))
    meta = {}
    for f in glob.glob(os.path.join(root, f"{w}_*", "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].replace("fury::(anonymous namespace)::", "").split("(")[0][-40:]
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            meta[k] = (r["VGPR_Count"], r["SGPR_Count"], r["LDS_Block_Size"])
    for k, cs in acc.items():
        if "fury" not in k and "kernel" not in k and "scan" not in k:
            continue
        vals = {c: sum(v) / len(v) for c, v in cs.items()}
        print(w, k, "vgpr/sgpr/lds", meta[k])
        print("   ", "  ".join(f"{c}={vals[c]:.4g}" for c in sorted(vals)))
