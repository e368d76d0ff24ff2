"""Kernel timeline of the last `steps` encoder steps of a bench trace: every dispatch with its HIP
stream, start and end relative to the first timed enc_mb_kernel (ms), to see what serialises.
usage: timeline.py <kernel_trace.csv> [steps] [filter-substring ...]"""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
flt = sys.argv[3:] or ['enc_mb_kernel', 'dec_parse_kernel', 'dec_recon_kernel', 'dec_hdr', 'dec_scan', 'enc_copy']
ks = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name'].split('(')[0].split('<')[0].replace('void ', '').replace('h264mi::', ''), r.get('Stream_Id', r.get('Queue_Id', '?')), r.get('Queue_Id', '?')) for r in rows)
mb = [k for k in ks if k[2] == 'enc_mb_kernel']
t0 = mb[-steps][0]
tend = max(k[1] for k in ks)
print(f'from first timed enc_mb_kernel to last kernel end: {(tend - t0) / 1e6:.2f} ms')
for s, e, n, st, q in ks:
    if e < t0 or not any(f in n for f in flt):
        continue
    print(f'{(s - t0) / 1e6:9.3f} {(e - t0) / 1e6:9.3f}  dur {(e - s) / 1e6:8.3f}  stream {st} queue {q}  {n}')
