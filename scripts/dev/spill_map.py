"""dev: per-loop MFMA / spill instruction counts of one kernel in a hipcc -S listing.
usage: python scripts/dev/spill_map.py file.s mangled_kernel_name"""
import re
import sys
from collections import defaultdict

s = open(sys.argv[1]).read()
name = sys.argv[2]
a = s.index(name + ':')
b = s.index('.Lfunc_end', a)
lines = s[a:b].split('\n')
cur = ('entry', 0)
stat = defaultdict(lambda: defaultdict(int))
for l in lines:
    m = re.match(r'^(\.LBB\d+_\d+):.*?(?:Header=(\S+) Depth=(\d+)|Parent Loop (\S+) Depth=(\d+)|Loop Header: Depth=(\d+))?', l)
    if m and l.startswith('.LBB'):
        lab = m.group(1)
        if 'Loop Header' in l:
            d = int(re.search(r'Depth=(\d+)', l).group(1))
            cur = (lab.replace('.L', ''), d)
        elif 'Header=' in l:
            hd = re.search(r'Header=(\S+) Depth=(\d+)', l)
            cur = (hd.group(1), int(hd.group(2)))
        elif 'Parent Loop' in l:
            hd = re.search(r'Parent Loop (\S+) Depth=(\d+)', l)
            cur = (hd.group(1) + '>', int(hd.group(2)))
        else:
            cur = ('straight', 0)
        continue
    t = l.strip()
    if not t or t.startswith(';') or t.startswith('.'):
        continue
    op = t.split()[0]
    st = stat[cur]
    st['insts'] += 1
    if op.startswith('v_mfma'):
        st['mfma'] += 1
    if op.startswith('scratch_store') or (op.startswith('buffer_store') and 'offen' in t and 's[0:3]' in t):
        st['spill_st'] += 1
    if op.startswith('scratch_load'):
        st['spill_ld'] += 1
    if op in ('v_writelane_b32',):
        st['sgpr_spill'] += 1
    if op in ('v_readlane_b32',):
        st['sgpr_fill'] += 1
for k, v in sorted(stat.items(), key=lambda x: -x[1]['mfma']):
    print(k, dict(v))
