"""Per (HIP stream, kernel) average duration over the timed region of a bench trace (the last
`steps` enc_mb_kernel launches).  usage: kstats_by_stream.py <kernel_trace.csv> [steps]"""
import csv, sys
from collections import defaultdict
rows = list(csv.DictReader(open(sys.argv[1])))
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 160
ks = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name'].split('(')[0].replace('h264mi::', ''), r['Stream_Id']) for r in rows)
mb = [k for k in ks if k[2] == 'enc_mb_kernel']
t0, t1 = mb[-steps][0], mb[-1][1]
print(f'timed region {(t1 - t0) / 1e6:.1f} ms = {(t1 - t0) / 1e6 / steps:.3f} ms per encoder step')
d = defaultdict(lambda: [0, 0])
for s, e, n, q in ks:
    if s >= t0 and e <= t1:
        d[(q, n)][0] += 1; d[(q, n)][1] += e - s
for (q, n), (c, t) in sorted(d.items()):
    print(f'stream {q} {n:28s} {c:5d} x avg {t / c / 1e3:9.1f} us   per step {t / steps / 1e3:8.1f} us')
