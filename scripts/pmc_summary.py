"""Summarise a rocprofv3 counter_collection.csv per kernel: dispatches and the
sum of every counter over them -> one CSV row per (kernel, counter)."""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(src, dst):
    files = glob.glob(os.path.join(src, '**', '*counter_collection.csv'), recursive=True)
    tot = defaultdict(float)
    disp = defaultdict(set)
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = row.get('Kernel_Name', '?')
                if len(k) > 90:
                    k = k[:90]
                tot[(k, row['Counter_Name'])] += float(row['Counter_Value'])
                disp[k].add(row.get('Dispatch_Id', ''))
    with open(dst, 'w', newline='') as fh:
        w = csv.writer(fh)
        w.writerow(['kernel', 'dispatches', 'counter', 'sum'])
        for (k, c), v in sorted(tot.items()):
            w.writerow([k, len(disp[k]), c, '%.6g' % v])
    print('summarised', len(files), 'files,', len(tot), 'rows ->', dst)


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2])
