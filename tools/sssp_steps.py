"""Summarise a GX_SSSP_VERBOSE=2 log (the last gx_sssp run in it) by step kind:
python tools/sssp_steps.py LOG [--all]"""
import re
import sys

L = [l for l in open(sys.argv[1]) if l.startswith('step')]
L = L[[i for i, l in enumerate(L) if l.startswith('step 0 ')][-1]:]
tot, cats = 0.0, {}
for l in L:
    mode, heavy, pull, us, items, edges = re.search(
        r'mode (\d) heavy (\d) pull (\d).*\| ([\d.]+) us items (\d+) edges (\d+)', l).groups()
    k = ('heavy-pull' if pull == '1' and heavy == '1' and mode == '3' else 'heavy' if mode == '3'
         else 'open' if mode != '0' else 'light')
    c = cats.setdefault(k, [0, 0, 0.0])
    c[0] += 1
    c[1] += int(edges)
    c[2] += float(us)
    tot += float(us)
    if '--all' in sys.argv:
        print(k, us, items, edges)
print(len(L), 'steps', round(tot), 'us;', {k: (v[0], v[1], round(v[2])) for k, v in cats.items()})
