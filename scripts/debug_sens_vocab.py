"""Dev tool (GPU box): SM-G-SUM sensitivity at small vocabularies, GPU vs the restatement oracle, with the
per-parameter-block worst relative error. usage: python scripts/debug_sens_vocab.py 63 127 255 999"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, 'nes-img-captioning_amd'))

import nicnes  # noqa: E402
from oracle import oracle as O  # noqa: E402
from oracle import sensitivity_ref as SR  # noqa: E402

NAMES = ['img_embed.weight', 'img_embed.bias', 'embed.weight', 'logit.weight', 'logit.bias', 'core.i2h.weight',
         'core.i2h.bias', 'core.h2h.weight', 'core.h2h.bias']
out = os.path.join(REPO, 'gpurun_out', 'sens_vocab')
os.makedirs(out, exist_ok=True)
for vocab in [int(v) for v in sys.argv[1:]]:
    for kind in ('wc', 'xavier'):
        dims = O.Dims(vocab_size=vocab)
        theta = O.make_theta(dims, 3, 4.0, 0.1) if kind == 'wc' else O.make_theta(dims, 0, 1.0, 0.0)
        rows = 12
        fc = np.random.Generator(np.random.PCG64(78)).standard_normal((rows, dims.F)).astype(np.float32)
        e = nicnes.Engine(vocab_size=vocab, max_batch=rows, max_members=2, noise_len=1 << 24, noise_seed=0)
        try:
            e.set_noise_table(O.noise_table(1 << 24, 123))
            e.set_theta(theta)
            e.set_df_table(np.zeros(0, np.uint64), np.zeros(0), np.log(64.0))
            e.set_batch(fc, [np.zeros((1, dims.T), np.int32)] * rows)
            raw = e.sum_sensitivity(rows).cpu().numpy()
            offs = list(e.offsets)
        finally:
            e.close()
        ref = SR.sum_sensitivity((dims.vocab_size + 1, dims.E, dims.R, dims.F), theta, fc, rows).numpy()
        np.savez(os.path.join(out, 'v%d_%s.npz' % (vocab, kind)), gpu=raw, ref=ref, offs=np.array(offs))
        print('vocab', vocab, kind, 'offsets', offs)
        for k, name in enumerate(NAMES):
            a, b = raw[offs[k]:offs[k + 1]].astype(np.float64), ref[offs[k]:offs[k + 1]].astype(np.float64)
            err = np.abs(a - b)
            rel = err / np.maximum(np.abs(b), 1e-30)
            big = np.abs(b) > 1e-3 * np.abs(ref).max()
            print('  %-18s n %8d max|ref| %.3e max abs err %.3e max rel (big) %.3e argmax %d' % (
                name, b.size, np.abs(b).max(), err.max(), rel[big].max() if big.any() else 0.0, int(err.argmax())))
        sys.stdout.flush()
