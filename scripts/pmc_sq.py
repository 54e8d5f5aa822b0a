#!/usr/bin/env python3
"""Per-kernel averages of SQ counters from a rocprofv3 --pmc counter_collection.csv
(summed over the dispatch's XCDs/SEs by rocprofv3; averaged over dispatches).

    python scripts/pmc_sq.py <counter_collection.csv> [kernel-substring]
"""
import collections
import csv
import sys


def main(path, pat=''):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(path)):
        k = r['Kernel_Name']
        if pat and pat not in k:
            continue
        acc[k][r['Counter_Name']].append(float(r['Counter_Value']))
    for k, cs in acc.items():
        print(k[:110])
        for c, v in sorted(cs.items()):
            print(f'   {c:28s} {sum(v) / len(v):16.1f}  (n={len(v)})')


if __name__ == '__main__':
    main(*sys.argv[1:])
