"""Time the decode variants (NICNES_DECODE=1 / 2) on the same workload in one process. Dev tool."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'nes-img-captioning_amd'))
import nicnes  # noqa: E402
import nicnes.synthetic as S  # noqa: E402

pop = int(os.environ.get('POP', '512'))
noise = torch.from_numpy(S.noise_table(1 << 27)).cuda()
eng, wl = {}, None
for v in ('2', '1'):
    os.environ['NICNES_DECODE'] = v
    e = nicnes.Engine(max_batch=128, max_members=pop, noise_len=1 << 27)
    if wl is None:
        wl = S.setup_engine_workload(e, B=128, noise=noise)
        keys, vals = nicnes.df_table_arrays(wl['df'])
    else:
        e.set_noise_table(noise)
        e.set_theta(wl['theta32'])
        e.set_df_table(keys, vals, np.log(float(wl['ref_len_raw'])))
        e.set_batch(wl['fc'], wl['gts'])
    e.set_timing(True)
    eng[v] = e
ref = None
for v, e in eng.items():
    f, s = e.evaluate(7, 0, 16, 0.01, return_seq=True)
    if ref is None:
        ref = (f, s)
    else:
        print('variant', v, 'tokens == variant 1:', bool(torch.equal(s, ref[1])), 'fitness:', bool(torch.equal(f, ref[0])))
res = {v: [] for v in eng}
for r in range(3):
    for v, e in eng.items():
        e.evaluate(r + 1, 0, pop, 0.01)
        res[v].append(e.kernel_times()[0])
for v in res:
    print('decode variant', v, 'median ms %.3f' % np.median(res[v]), 'fallbacks', eng[v].stats())
