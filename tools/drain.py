"""Timeline of the last K frame steps of a bench run from a rocprofv3 kernel trace: when the encoder's
last frame ended, when each parse / reconstruction launch of the tail ran (ms from the start of the
K-th-last enc_mb_kernel).  usage: drain.py <run_kernel_trace.csv> [K]"""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
K = int(sys.argv[2]) if len(sys.argv) > 2 else 20
ev = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name'].split('(')[0].split('<')[0].replace('void ', '').replace('h264mi::', '')) for r in rows)
enc = [e for e in ev if e[2] == 'enc_mb_kernel']
t0 = enc[-K][0]
ms = lambda t: (t - t0) / 1e6
print(f'encoder: {K} frames from 0 to {ms(enc[-1][1]):.2f} ms ({(enc[-1][1] - enc[-K][0]) / 1e6 / K:.2f} ms per frame step)')
for s, e, n in ev:
    if e >= t0 and n in ('dec_scan_kernel', 'dec_hdr_kernel', 'dec_parse_kernel', 'dec_recon_kernel'):
        print(f'{n:18s} {ms(s):8.2f} -> {ms(e):8.2f}  ({(e - s) / 1e6:.2f} ms)')
