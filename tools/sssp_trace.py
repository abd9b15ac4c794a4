"""Per-launch view of one gx_sssp run from a rocprofv3 --kernel-trace CSV:
python tools/sssp_trace.py TRACE.csv  (the last k_sssp_init onwards)."""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ks = [r for r in rows if 'k_sssp' in r['Kernel_Name']]
ks = ks[max(i for i, r in enumerate(ks) if 'k_sssp_init' in r['Kernel_Name']):]
tot, seq = {}, []
for r in ks:
    d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
    n = re.search(r'k_sssp_\w+', r['Kernel_Name']).group(0)
    tot[n] = tot.get(n, 0) + d
    if n in ('k_sssp_relax', 'k_sssp_advance'):
        seq.append('%s%d' % (n[7], round(d)))
print({k: round(v) for k, v in tot.items()})
print(' '.join(seq))
print('span us', (int(ks[-1]['End_Timestamp']) - int(ks[0]['Start_Timestamp'])) / 1e3)
