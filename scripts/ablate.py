"""Decode-kernel ablation: time timing-only builds (make -C nes-img-captioning_amd ablate) in ONE
process on ONE GPU, interleaved rounds (cdna_hip_programming.md 5.4 rule 24). Dev tool."""
import glob
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'nes-img-captioning_amd'))
import nicnes  # noqa: E402
import nicnes.synthetic as S  # noqa: E402


def main():
    pop = int(os.environ.get('POP', '512'))
    rounds = int(os.environ.get('ROUNDS', '3'))
    libs = sorted(glob.glob(os.path.join(REPO, 'nes-img-captioning_amd', 'build', 'ablate', 'libnicnes_*.so')))
    noise = torch.from_numpy(S.noise_table(1 << 27)).cuda()
    engines = {}
    libs.sort(key=lambda p: not p.endswith('_base.so'))          # base first: it makes the refs
    wl = None
    for path in libs:
        name = os.path.basename(path)[len('libnicnes_'):-3]
        e = nicnes.Engine(max_batch=128, max_members=pop, noise_len=1 << 27, lib_path=path)
        if wl is None:
            wl = S.setup_engine_workload(e, B=128, noise=noise)
            keys, vals = nicnes.df_table_arrays(wl['df'])
        else:                                   # timing-only builds decode garbage: reuse base's refs
            e.set_noise_table(noise)
            e.set_theta(wl['theta32'])
            e.set_df_table(keys, vals, np.log(float(wl['ref_len_raw'])))
            e.set_batch(wl['fc'], wl['gts'])
        e.set_timing(True)
        engines[name] = e
    res = {k: [] for k in engines}
    for r in range(rounds):
        for k, e in engines.items():
            e.evaluate(r + 1, 0, pop, 0.01)
            res[k].append(e.kernel_times()[0])
    ref = engines['base'].evaluate(99, 0, 8, 0.01, return_seq=True)
    for k in [x for x in os.environ.get('EXACT', '').split(',') if x]:   # variants that must match base
        if k in engines:
            got = engines[k].evaluate(99, 0, 8, 0.01, return_seq=True)
            print(k, 'tokens == base:', bool(torch.equal(got[1], ref[1])), 'fitness == base:',
                  bool(torch.equal(got[0], ref[0])))
    for k in [x for x in engines if x.startswith('prof')]:   # DECODE_PROF builds: section cycles
        _, seq = engines[k].evaluate(50, 0, pop, 0.01, return_seq=True)
        cyc = seq.view(pop, -1)[:, :128].reshape(pop, 8, 16).double().cpu().numpy()   # [member, wave, section]
        names = ['img', 'embed', 'cell_p1', 'cell_p2', 'cell_elem', 'logit', 'finish', 'tail', 'lg_issue',
                 'lg_mfma_epi', 'lg_store_or_wait', 'lg_barrier', 'lg_form', 's13', 's14', 's15']
        tot = cyc.sum(axis=2).mean()
        print(k, 'mean cycles per wave:', json.dumps({n: round(float(cyc[:, :, i].mean()), 0) for i, n in enumerate(names)}),
              'total', round(float(tot), 0), 'frac', json.dumps({n: round(float(cyc[:, :, i].mean() / tot), 4)
                                                                   for i, n in enumerate(names)}))
        for i in (5, 8, 9, 10, 11, 12):
            print(k, names[i], 'sgn0 %.0f sgn1 %.0f' % (cyc[:, :4, i].mean(), cyc[:, 4:, i].mean()))
    base = np.median(res['base'])
    out = {k: {'median_ms': round(float(np.median(v)), 3), 'min_ms': round(float(np.min(v)), 3),
               'vs_base': round(float(np.median(v) / base), 3)} for k, v in res.items()}
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main()
