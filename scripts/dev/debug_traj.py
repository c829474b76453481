"""debug: master trajectory GPU vs oracle engine (dev helper)"""
import sys
import numpy as np
sys.path.insert(0, '.'); sys.path.insert(0, 'nes-img-captioning_amd')
from tests.test_gpu_master import _Loader, _spec
from tests.cpu_engine import OracleEngine
import nicnes
import nicnes.synthetic as S
from nicnes import master as M
from oracle import oracle as O
dims = O.Dims()
theta = O.make_theta(dims, 0, 4.0, 0.1)
fc = np.random.Generator(np.random.PCG64(1234)).standard_normal((16, dims.F)).astype(np.float32)
base, _, _ = O.decode(dims, theta, fc)
gts, df, n = S.build_references(base, dims.vocab_size, seed=9, n_refs=5, df_sets=128)
table = O.noise_table(1 << 23, 123)
for maxb in (8, 16):
    e = nicnes.Engine(max_batch=maxb, max_members=4, noise_len=1 << 23, noise_seed=0)
    e.set_noise_table(table)
    k, v = nicnes.df_table_arrays(df)
    e.set_df_table(k, v, np.log(float(n)))
    gpu = M.EngineMaster(_spec(4), e, theta=theta)
    ora_e = OracleEngine(dims, theta, fc, gts, df, n, table, noise_seed=0)
    ora = M.EngineMaster(_spec(4), ora_e, theta=theta)
    gpu.run(_Loader(fc, gts), max_iterations=3)
    ora.run(_Loader(fc, gts), max_iterations=3)
    for a, b in zip(gpu.stats, ora.stats):
        print(maxb, a['iter'], a['score_mean'], b['score_mean'], a['noise_stdev'], b['noise_stdev'], a['update_ratio'], b['update_ratio'])
    print('theta rel', np.abs(e.theta()[0].cpu().numpy() - ora_e.adam.theta).max())
    e.close()
