"""A/B helper: `python scripts/bench_tuned.py key=value[,key=value] <bench.py args>` sets library
tuning knobs (fury_set_tuning) and runs bench.py's main in the same process."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from fury_amd import _native as N  # noqa: E402

if __name__ == "__main__":
    for kv in sys.argv[1].split(","):
        if kv:
            k, v = kv.split("=")
            assert N.lib().fury_set_tuning(k.encode(), int(v)) == 0, N.last_error()
    sys.argv = [sys.argv[0]] + sys.argv[2:]
    bench.main()
