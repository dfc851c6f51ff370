"""A/B: decode_batch wall time with sizing="measure" (decode sizing pass + host sync) vs
"bound" (outputs sized from the row bytes, one pass, one host read to trim)."""
import sys, time, torch
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from fury_amd.encoder import Encoders, column_to_device
from fury_amd.workloads import SCHEMAS, gen_columns
dev = torch.device("cuda:0")
for name, n in (("mixed", 2_000_000), ("nested", 1_000_000)):
    fields = SCHEMAS[name]
    cols = [column_to_device(c, dev) for c in gen_columns(name, fields, n, seed=5)]
    enc = Encoders.bean(fields, device=dev)
    b = enc.encode_batch(cols, n)
    for s in ("measure", "bound") * 2:
        enc.decode_batch(b, sizing=s); torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(10):
            enc.decode_batch(b, sizing=s)
        torch.cuda.synchronize()
        print(name, n, s, round((time.perf_counter() - t) / 10 * 1e3, 3), "ms per decode_batch", flush=True)
