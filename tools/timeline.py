"""Overlap analysis of a rocprofv3 kernel trace (the bench's timed region): per kernel name the busy
time, and for the last N ms of the trace how much of the wall time had each kernel running and how
much had >= 2 of the codec kernels running at once.   usage: timeline.py <trace.csv> [window_ms]"""
import csv, sys
from collections import defaultdict

rows = []
for r in csv.DictReader(open(sys.argv[1])):
    n = r['Kernel_Name']
    if 'h264mi::' not in n:
        continue
    rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), n.split('h264mi::')[1].split('(')[0]))
rows.sort()
end = max(e for _, e, _ in rows)
win = float(sys.argv[2]) if len(sys.argv) > 2 else 500.0
t0 = end - win * 1e6
rows = [(max(s, t0), e, n) for s, e, n in rows if e > t0]
ev = []
for s, e, n in rows:
    ev.append((s, 1, n)); ev.append((e, -1, n))
ev.sort()
active = defaultdict(int)
busy = defaultdict(float)
multi = 0.0
anyb = 0.0
last = t0
for t, d, n in ev:
    dt = t - last
    names = [k for k, v in active.items() if v > 0]
    for k in names:
        busy[k] += dt
    if names:
        anyb += dt
    if len(names) >= 2:
        multi += dt
    active[n] += d
    last = t
W = end - t0
print(f'window {W / 1e6:.1f} ms: any kernel {anyb / W:.1%}, >=2 kernels {multi / W:.1%}')
for k, v in sorted(busy.items(), key=lambda kv: -kv[1]):
    print(f'  {k:28s} running {v / W:6.1%} of wall')
