"""Summarise a gfx950 .s by basic block: instruction-class counts (dev tool)."""
import re
import sys
from collections import Counter, OrderedDict

def classify(op):
    if op.startswith('v_mfma'): return 'mfma'
    if op.startswith('ds_read') or op.startswith('ds_load'): return 'ds_r'
    if op.startswith('ds_write') or op.startswith('ds_store') or op.startswith('ds_'): return 'ds_w'
    if op.startswith('buffer_load') or op.startswith('global_load'): return 'vmem_r'
    if op.startswith('buffer_store') or op.startswith('global_store'): return 'vmem_w'
    if op.startswith('scratch_'): return 'scratch'
    if op in ('v_exp_f32', 'v_log_f32', 'v_rcp_f32', 'v_sqrt_f32') or op.startswith(('v_exp', 'v_log', 'v_rcp')): return 'trans'
    if op.startswith('v_'): return 'valu'
    if op.startswith('s_waitcnt'): return 'wait'
    if op.startswith('s_barrier'): return 'barrier'
    if op.startswith('s_'): return 'salu'
    return 'other'

blocks = OrderedDict(); cur = 'entry'; blocks[cur] = Counter()
for line in open(sys.argv[1]):
    line = line.split(';')[0].rstrip()
    if not line.strip(): continue
    m = re.match(r'^(\.LBB\w+|\w+):', line)
    if m:
        cur = m.group(1); blocks.setdefault(cur, Counter()); continue
    if line.startswith('\t.') or line.startswith('.'): continue
    op = line.split()[0]
    blocks[cur][classify(op)] += 1
minm = int(sys.argv[2]) if len(sys.argv) > 2 else 1
for k, c in blocks.items():
    if c['mfma'] >= minm:
        print(k, dict(c))
