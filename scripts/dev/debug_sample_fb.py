"""Dev: sampled picks at the bench shape (B = 128 images x 5 rows, P members) with the stage-record scan vs the
full walk (NICNES_FORCE_EXACT=1): fallback counts and token agreement."""
import os
import sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..', 'nes-img-captioning_amd'))
import torch  # noqa: E402
import nicnes  # noqa: E402
import nicnes.synthetic as S  # noqa: E402

P = int(sys.argv[1]) if len(sys.argv) > 1 else 32
noise = torch.from_numpy(S.noise_table(1 << 27)).cuda()
res = {}
for force in ('0', '1'):
    os.environ['NICNES_FORCE_EXACT'] = force
    e = nicnes.Engine(max_batch=640, max_members=P, noise_len=1 << 27, lib_path=os.environ.get('LIB') or None)
    S.setup_engine_workload(e, B=128, noise=noise)
    e.set_fitness_mode('sample')
    e.set_rows_per_image(5)
    b0 = e.stats()['sample_stage_fallbacks']
    fit, seq, lp = e.evaluate(3, 0, P, 0.01, return_seq=True, return_lp=True)
    res[force] = (seq.cpu().numpy(), lp.cpu().numpy(), e.stats()['sample_stage_fallbacks'] - b0)
    e.close()
(s0, l0, f0), (s1, l1, f1) = res['0'], res['1']
diff = np.argwhere(s0 != s1)
print('fallbacks scan %d full %d; token mismatches %d of %d' % (f0, f1, diff.shape[0], s0.size))
for d in diff[:10]:
    m, sg, r, t = d
    print('member %d sign %d row %d step %d: scan %d full %d  (scan id %% 64 = %d)' % (m, sg, r, t, s0[m, sg, r, t],
                                                                                  s1[m, sg, r, t], s0[m, sg, r, t] % 64))
