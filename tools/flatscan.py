"""Counts flat_* memory instructions per kernel / device function in gfx950 assembly, to find
accesses whose address space the compiler could not prove ("Address spaces").

    hipcc -O3 -std=c++17 --offload-arch=gfx950 -x hip --cuda-device-only -S \\
        fury_amd/csrc/levels.hip -I fury_amd/csrc -o /tmp/levels.s
    python tools/flatscan.py /tmp/levels.s
"""
import collections
import re
import sys


def scan(path):
    cur, cnt = None, collections.Counter()
    for line in open(path):
        m = re.match(r"^(_Z[^:\s]+):", line)
        if m:
            cur = m.group(1)
            continue
        if cur and re.match(r"\s+flat_(load|store|atomic)", line):
            cnt[cur] += 1
    return cnt


if __name__ == "__main__":
    for f in sys.argv[1:]:
        for name, n in scan(f).most_common():
            print(f"{f.split('/')[-1]}\t{n}\t{name}")
