"""Per-basic-block instruction counts of one kernel in a hipcc -S listing:
python scripts/isa_blocks.py listing.s <mangled-name-substring>"""
import re
import sys

lines = open(sys.argv[1]).read().split('\n')
key = sys.argv[2]
st = [i for i, l in enumerate(lines) if re.match(r'^_Z\S*:', l) and key in l][0]
en = [i for i in range(st, len(lines)) if lines[i].startswith('.Lfunc_end')][0]
blocks, cur = [], None
for l in lines[st:en]:
    m = re.match(r'^(\.LBB\S+):', l)
    if m:
        cur = [m.group(1), []]
        blocks.append(cur)
        continue
    t = l.strip()
    if not t or t.startswith(';') or t.startswith('.'):
        continue
    if cur is None:
        cur = ['entry', []]
        blocks.append(cur)
    cur[1].append(t)
tot = {}
for nm, ins in blocks:
    c = {k: sum(1 for x in ins if x.startswith(k)) for k in ('v_', 's_', 'ds_', 'buffer_', 'global_')}
    br = [x for x in ins if 's_cbranch' in x or 's_branch' in x]
    print(nm, len(ins), ' '.join(f'{k}{v}' for k, v in c.items() if v), '|', br[-1] if br else '')
    for k, v in c.items():
        tot[k] = tot.get(k, 0) + v
print('total', tot)
