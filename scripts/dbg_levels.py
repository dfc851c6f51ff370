"""DEBUG: first mismatching entry of a nested column between the level engine (nested_decode 1),
the row walk (2) and the oracle (tests/test_device.py _engine_schemas)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from fury_amd import _native as N
    from fury_amd.beans import beans_to_columns
    from fury_amd.encoder import Encoders, column_to_host
    from oracle import oracle as O
    from tests.test_device import _dev_cols, _engine_schemas, _random_value
    name = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 3001
    fields = _engine_schemas()[name]
    rng = np.random.default_rng(len(name) * 7)
    beans = [{f.name: _random_value(f, rng) for f in fields} for _ in range(n)]
    host = beans_to_columns(fields, beans)
    dev = torch.device("cuda:0")
    enc = Encoders.bean(fields, device=dev)
    batch = enc.encode_batch(_dev_cols(host, dev), n)
    want, offs = O.encode(fields, host, n)
    ref = O.decode(fields, want, offs, n)
    outs = {}
    for mode in (1, 2):
        N.lib().fury_set_tuning(b"nested_decode", mode)
        outs[mode] = [column_to_host(c) for c in enc.decode_batch(batch)]

    def walk(fs, cols_by, path):
        for k, f in enumerate(fs):
            cs = {m: c[k] for m, c in cols_by.items()}
            p = path + f.name
            for attr in ("offsets", "validity", "values"):
                arrs = {m: getattr(c, attr) for m, c in cs.items()}
                if any(a is None for a in arrs.values()):
                    continue
                a = {m: np.asarray(v).view(np.uint8) for m, v in arrs.items()}
                L = min(len(x) for x in a.values())
                for m in (0, 1):
                    d = np.nonzero(a[m][:L] != a["ref"][:L])[0]
                    if len(d):
                        print(p, attr, "mode", m, "first diff byte", d[0], "of", L,
                              a[m][max(d[0] - 8, 0):d[0] + 8], a["ref"][max(d[0] - 8, 0):d[0] + 8])
            if f.children and all(c.child for c in cs.values()):
                walk(f.children, {m: c.child for m, c in cs.items()}, p + ".")

    walk(fields, {1: outs[1], 2: outs[2], "ref": ref}, "")
    print("done")


if __name__ == "__main__":
    main()
