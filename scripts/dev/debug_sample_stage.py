"""Dev: sampled picks with the stage scan vs the full walk (NICNES_FORCE_EXACT=1) on a small batch; prints the
share of picks that are a stage's last id and the fallback counters."""
import os
import sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..', 'nes-img-captioning_amd'))
import torch  # noqa: E402
import nicnes  # noqa: E402
import nicnes.synthetic as S  # noqa: E402
from oracle import oracle as O  # noqa: E402

NL = 1 << 23
dims = O.Dims()
theta = O.make_theta(dims, 0, 4.0, 0.1)
B = 40
fc = np.random.Generator(np.random.PCG64(5)).standard_normal((B, dims.F)).astype(np.float32)
u = np.random.Generator(np.random.PCG64(6)).random((1, 2, B, dims.T))
table = O.noise_table(NL, 123)
res = {}
for force in ('0', '1'):
    os.environ['NICNES_FORCE_EXACT'] = force
    e = nicnes.Engine(max_batch=B, max_members=2, noise_len=NL, noise_seed=7)
    e.set_noise_table(table)
    base, _, _ = O.decode(dims, theta, fc)
    gts, df, n = S.build_references(base, dims.vocab_size, seed=1, df_sets=64)
    e.set_theta(theta)
    k, v = nicnes.df_table_arrays(df)
    e.set_df_table(k, v, np.log(float(n)))
    e.set_batch(fc, gts)
    e.set_fitness_mode('sample')
    e.set_sample_draws(u)
    _, seq, lp = e.evaluate(1, 0, 1, 0.0, return_seq=True, return_lp=True)
    seq = seq.cpu().numpy()
    res[force] = seq
    print('force', force, 'last-id share', float(np.mean((seq % 64) == 63)), 'stats', e.stats())
    e.close()
oseq, olp, ofr = O.decode_sample(dims, theta, fc, u[0, 0])
print('scan == full', np.array_equal(res['0'], res['1']))
print('full vs oracle row0', res['1'][0, 0, 0], oseq[0])
print('scan vs oracle row0', res['0'][0, 0, 0], oseq[0])
