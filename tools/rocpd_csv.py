"""Convert a rocprofv3 SQLite result (`run_results.db`, the default output format of this ROCm's
rocprofv3) into the kernel-trace CSV columns tools/drain.py and tools/timeline.py read, plus a
kernel_stats.csv like `--stats` writes (Name, Calls, AverageNs, TotalDurationNs, Percentage).
usage: rocpd_csv.py <run_results.db> <out_dir>"""
import csv, os, sqlite3, sys
from collections import defaultdict

db, out = sys.argv[1], sys.argv[2]
os.makedirs(out, exist_ok=True)
c = sqlite3.connect(db)
rows = c.execute('select name, start, end, stream_id, queue_id, grid_x, workgroup_x from kernels order by start').fetchall()
with open(os.path.join(out, 'run_kernel_trace.csv'), 'w', newline='') as f:
    w = csv.writer(f)
    w.writerow(['Kernel_Name', 'Start_Timestamp', 'End_Timestamp', 'Stream_Id', 'Queue_Id', 'Grid_Size_X', 'Workgroup_Size_X'])
    w.writerows(rows)
agg = defaultdict(lambda: [0, 0])
for n, s, e, *_ in rows:
    agg[n][0] += 1
    agg[n][1] += e - s
tot = sum(v[1] for v in agg.values()) or 1
with open(os.path.join(out, 'run_kernel_stats.csv'), 'w', newline='') as f:
    w = csv.writer(f)
    w.writerow(['Name', 'Calls', 'TotalDurationNs', 'AverageNs', 'Percentage'])
    for n, (k, t) in sorted(agg.items(), key=lambda x: -x[1][1]):
        w.writerow([n, k, t, t / k, 100.0 * t / tot])
print(f'{len(rows)} dispatches -> {out}')
