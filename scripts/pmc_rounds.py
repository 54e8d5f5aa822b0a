#!/usr/bin/env python3
"""Per-dispatch SQ counters of one kernel from a rocprofv3 --pmc
counter_collection.csv: the dispatches sorted by SQ_INSTS_VALU, and the
per-wave averages over the top half (the solve rounds of an online run).

    python scripts/pmc_rounds.py <counter_collection.csv> <kernel-substring>
"""
import collections
import csv
import sys


def main(path, pat):
    disp = collections.defaultdict(dict)
    for r in csv.DictReader(open(path)):
        if pat not in r['Kernel_Name']:
            continue
        d = disp[r.get('Dispatch_Id', r.get('Correlation_Id'))]
        d[r['Counter_Name']] = d.get(r['Counter_Name'], 0.0) + float(r['Counter_Value'])
    rows = sorted(disp.values(), key=lambda d: d.get('SQ_INSTS_VALU', 0.0))
    top = rows[len(rows) // 2:]
    print(f'{len(rows)} dispatches of {pat}; averages over the top {len(top)} by SQ_INSTS_VALU:')
    keys = sorted({k for d in top for k in d})
    w = sum(d.get('SQ_WAVES', 0.0) for d in top) / max(len(top), 1)
    for k in keys:
        v = sum(d.get(k, 0.0) for d in top) / len(top)
        print(f'   {k:24s} {v:16.1f}' + (f'   per wave {v / w:12.1f}' if w and k != 'SQ_WAVES' else ''))


if __name__ == '__main__':
    main(*sys.argv[1:])
