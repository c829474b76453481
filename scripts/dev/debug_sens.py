"""Dev: the SM-G-SUM vector per parameter segment, new kernels vs the old rocBLAS build vs the torch oracle."""
import os
import sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..', 'nes-img-captioning_amd'))
import nicnes  # noqa: E402
from oracle import oracle as O  # noqa: E402
from oracle import sensitivity_ref as SR  # noqa: E402

NL = 1 << 23
rows = int(sys.argv[1]) if len(sys.argv) > 1 else 41
dims = O.Dims()
theta = O.make_theta(dims, 3, 4.0, 0.1)
fc = np.random.Generator(np.random.PCG64(77)).standard_normal((rows + 4, dims.F)).astype(np.float32)
out = {}
for name, lib in (('new', None), ('old', 'ablate_libs/libnicnes_oldsens.so')):
    e = nicnes.Engine(max_batch=rows + 4, max_members=2, noise_len=NL, noise_seed=0, lib_path=lib)
    e.set_noise_table(O.noise_table(NL, 123))
    e.set_theta(theta)
    e.set_df_table(np.zeros(0, np.uint64), np.zeros(0), np.log(64.0))
    e.set_batch(fc, [np.zeros((1, dims.T), np.int32)] * fc.shape[0])
    out[name] = e.sum_sensitivity(rows).cpu().numpy().astype(np.float64)
    offs = e.offsets
    e.close()
ref = SR.sum_sensitivity((dims.vocab_size + 1, dims.E, dims.R, dims.F), theta, fc[:rows], rows).numpy().astype(np.float64)
names = ['img_w', 'img_b', 'emb', 'log_w', 'log_b', 'i2h_w', 'i2h_b', 'h2h_w', 'h2h_b']
offs = list(offs)
big = 1e-3 * np.abs(ref).max()
for q, nm in enumerate(names):
    a, b = offs[q], offs[q + 1]
    r = ref[a:b]
    for k in ('new', 'old'):
        g = out[k][a:b]
        m = np.abs(r) > big
        rel = (np.abs(g - r) / np.maximum(np.abs(r), 1e-30))[m]
        i = int(np.argmax(np.abs(g - r)))
        print('%-6s %-4s max rel %.3g (n=%d)  worst abs at %d: got %.6g ref %.6g' % (
            nm, k, rel.max() if rel.size else 0.0, m.sum(), i, g[i], r[i]))
print('new vs old max rel', float((np.abs(out['new'] - out['old']) / np.maximum(np.abs(out['old']), 1e-30))[np.abs(ref) > big].max()))
