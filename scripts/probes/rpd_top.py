"""Top kernels of a rocprofv3 SQLite (rocpd) result: name, calls, total ms, avg us.

    python scripts/probes/rpd_top.py gpurun_out/prof_ts [N]
"""
import glob
import os
import sqlite3
import sys

d = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 15
db = sqlite3.connect(sorted(glob.glob(os.path.join(d, '**', '*.db'), recursive=True))[-1])
for name, calls, tot, avg, pct in db.execute('select * from top_kernels limit %d' % n):
    short = name.replace('(anonymous namespace)::', '').split('(')[0][-60:]
    print('%-60s %6d %10.2f ms %9.2f us %5.1f%%' % (short, calls, tot / 1e3, avg, pct))
