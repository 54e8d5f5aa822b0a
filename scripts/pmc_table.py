#!/usr/bin/env python3
"""Per-kernel average of every rocprofv3 PMC counter found under the given
directories (one directory per --pmc pass), plus derived figures:
HBM bytes (FETCH_SIZE x2 per MI355X_MICROARCH.md's gfx950 correction +
WRITE_SIZE), VALU instructions per wave and the stall split.

    python scripts/pmc_table.py gpurun_out/pmc_TAG_1 gpurun_out/pmc_TAG_2 ...
"""
import collections
import csv
import os
import sys


def main(dirs):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for d in dirs:
        for root, _, files in os.walk(d):
            for fn in files:
                if fn.endswith('counter_collection.csv'):
                    for r in csv.DictReader(open(os.path.join(root, fn))):
                        acc[r['Kernel_Name']][r['Counter_Name']].append(float(r['Counter_Value']))
                if fn.endswith('kernel_trace.csv'):
                    for r in csv.DictReader(open(os.path.join(root, fn))):
                        dur[r['Kernel_Name']].append(float(r['End_Timestamp']) - float(r['Start_Timestamp']))
    for k in sorted(acc, key=lambda k: -sum(dur.get(k, [0]))):
        c = {n: sum(v) / len(v) for n, v in acc[k].items()}
        name = k if len(k) < 90 else k[:87] + '...'
        d = dur.get(k)
        print(f'== {name}  (avg {sum(d) / len(d) / 1e3:.1f} us over {len(d)} dispatches)' if d else f'== {name}')
        for n in sorted(c):
            print(f'   {n:28s} {c[n]:.4g}')
        if 'FETCH_SIZE' in c or 'WRITE_SIZE' in c:
            b = 2 * 1024 * c.get('FETCH_SIZE', 0) + 1024 * c.get('WRITE_SIZE', 0)
            print(f'   {"HBM bytes/launch (x2 fetch)":28s} {b:.4g}')
        if 'SQ_WAVES' in c and 'SQ_INSTS_VALU' in c:
            print(f'   {"VALU instr / wave":28s} {c["SQ_INSTS_VALU"] / max(c["SQ_WAVES"], 1):.4g}')
        if 'SQ_WAVE_CYCLES' in c:
            wc = c['SQ_WAVE_CYCLES']
            for n in ('SQ_WAIT_ANY', 'SQ_WAIT_INST_ANY', 'SQ_ACTIVE_INST_VALU', 'SQ_ACTIVE_INST_ANY'):
                if n in c:
                    print(f'   {n + " / wave cycles":28s} {c[n] / max(wc, 1):.3f}')


if __name__ == '__main__':
    main(sys.argv[1:])
