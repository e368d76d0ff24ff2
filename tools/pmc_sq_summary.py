"""Summarise an SQ counter pass (tools/pmc_sq.sh): per kernel, the averages per dispatch and the
wave-cycle split parked (s_waitcnt / barrier) / issue-stalled / issuing."""
import csv, glob, sys
from collections import defaultdict

d = sys.argv[1]
f = glob.glob(f'{d}/**/*counter_collection.csv', recursive=True)[0]
acc = defaultdict(lambda: defaultdict(float))
disp = defaultdict(set)
for r in csv.DictReader(open(f)):
    k = r['Kernel_Name'].split('(')[0][:48]
    acc[k][r['Counter_Name']] += float(r['Counter_Value'])
    disp[k].add(r['Dispatch_Id'])
for k, c in sorted(acc.items(), key=lambda kv: -kv[1].get('SQ_WAVE_CYCLES', 0)):
    n = len(disp[k])
    wc = c.get('SQ_WAVE_CYCLES', 0) or 1
    print(f"{k:48s} disp {n:4d} wave-cyc/disp {wc / n:12.0f}  parked {c.get('SQ_WAIT_ANY', 0) / wc:5.1%} "
          f"stall {c.get('SQ_WAIT_INST_ANY', 0) / wc:5.1%} active {c.get('SQ_ACTIVE_INST_ANY', 0) / wc:5.1%}  "
          f"valu/disp {c.get('SQ_INSTS_VALU', 0) / n:11.0f} salu {c.get('SQ_INSTS_SALU', 0) / n:11.0f} "
          f"lds {c.get('SQ_INSTS_LDS', 0) / n:10.0f} smem {c.get('SQ_INSTS_SMEM', 0) / n:9.0f}")
