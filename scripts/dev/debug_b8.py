"""debug: small-batch evaluate vs oracle across decode shapes (dev helper)"""
import sys
import numpy as np
sys.path.insert(0, '.'); sys.path.insert(0, 'nes-img-captioning_amd')
import torch
import nicnes
import nicnes.synthetic as S
from oracle import oracle as O, cider_ref as CR
dims = O.Dims()
theta = O.make_theta(dims, 0, 4.0, 0.1)
fc = np.random.Generator(np.random.PCG64(1234)).standard_normal((16, dims.F)).astype(np.float32)
base, _, _ = O.decode(dims, theta, fc)
gts, df, n = S.build_references(base, dims.vocab_size, seed=9, n_refs=5, df_sets=128)
table = O.noise_table(1 << 23, 123)
e = nicnes.Engine(max_batch=8, max_members=4, noise_len=1 << 23, noise_seed=0)
e.set_noise_table(table)
k, v = nicnes.df_table_arrays(df)
e.set_df_table(k, v, np.log(float(n)))
e.set_theta(theta)
scorer = CR.CiderDOracle(df, n)
for B in (8, 16):
    e.set_batch(fc[:B], gts[:B])
    for shape in ((0, 0), (1, 4), (16, 2), (4, 2), (1, 2), (16, 4)):
        e.set_decode_split(*shape)
        fit, seq = e.evaluate(1, 0, 4, 0.005, return_seq=True)
        fit, seq = fit.cpu().numpy(), seq.cpu().numpy()
        bad = []
        for m in range(4):
            idx = O.noise_index(0, 1, m, 1 << 23, dims.D)
            for s, sg in enumerate((1, -1)):
                oseq, _, fr = O.decode(dims, O.perturb(theta, table, idx, 0.005, sg), fc[:B])
                f_ref = CR.rollout_fitness(scorer, oseq, gts[:B])[0]
                if not np.array_equal(oseq, seq[m, s]) or abs(f_ref - fit[m, s]) > 1e-9 * f_ref:
                    bad.append((m, s, int((oseq != seq[m, s]).any(1).sum()), fit[m, s], f_ref))
        print('B', B, 'shape', shape, e.decode_shape(B, 4), 'bad', bad[:3], flush=True)
