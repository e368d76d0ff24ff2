"""Per-queue busy time and idle gaps of a rocprofv3 kernel trace (timed region = last window ms).
usage: queue_gaps.py <kernel_trace.csv> [window_ms]"""
import csv, sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
win = float(sys.argv[2]) if len(sys.argv) > 2 else 400.0
qk = 'Stream_Id' if 'Stream_Id' in rows[0] else 'Queue_Id'
ks = []
for r in rows:
    n = r['Kernel_Name'].split('(')[0].replace('h264mi::', '')[:28]
    ks.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), n, r[qk]))
end = max(e for _, e, _, _ in ks)
t0 = end - win * 1e6
byq = defaultdict(list)
for s, e, n, q in ks:
    if e > t0:
        byq[q].append((max(s, t0), e, n))
for q, L in byq.items():
    L.sort()
    busy = sum(e - s for s, e, _ in L)
    gaps = defaultdict(lambda: [0, 0.0])  # gap before kernel name
    for (s0, e0, n0), (s1, e1, n1) in zip(L, L[1:]):
        g = max(0, s1 - e0)
        gaps[n1][0] += 1; gaps[n1][1] += g
    names = sorted(set(n for _, _, n in L))
    print(f'{qk} {q}: {len(L)} kernels, busy {busy / (win * 1e6):.1%} of {win:.0f} ms; kernels: {", ".join(names)}')
    for n, (c, g) in sorted(gaps.items(), key=lambda kv: -kv[1][1]):
        print(f'    idle before {n:28s} {c:5d} x avg {g / max(c, 1) / 1e3:8.1f} us  total {g / 1e6:7.2f} ms')
