"""Print the kernel_stats.csv written by rocprofv3 --stats (searched under the given directory)."""
import csv, glob, os, sys

d = sys.argv[1]
files = glob.glob(os.path.join(d, '**', '*kernel_stats.csv'), recursive=True)
if not files:
    sys.exit(f'no kernel_stats.csv under {d}')
for f in files:
    print(f)
    rows = list(csv.DictReader(open(f)))
    for r in rows:
        name = r['Name'].split('(')[0][:60]
        print(f"{name:60s} calls {r['Calls']:>6s} avg {float(r['AverageNs'])/1e3:10.1f} us  total {float(r['TotalDurationNs'])/1e6:9.2f} ms  {float(r['Percentage']):6.2f}%")
