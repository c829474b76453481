"""Dev tool (GPU box): how much decode work a theta leaves after the early exit. A workgroup (member slab) runs
steps until every row of both signs has emitted the end token (nets.py:242-243); the logit steps it runs are
1 + the largest caption length over its rows (capped at T). Prints, for the bench workload at xavier theta and at the
peaked trained-like theta (--theta-gain 4 --bias-std 0.1), the mean logit steps per workgroup and the share of
the 16-step maximum, so two bench lines' members/s can be compared per unit of work.
usage: python scripts/decode_work.py [P]"""
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'nes-img-captioning_amd'))
import nicnes  # noqa: E402
import nicnes.synthetic as S  # noqa: E402

P = int(sys.argv[1]) if len(sys.argv) > 1 else 512
noise = torch.from_numpy(S.noise_table(1 << 27)).cuda()
out = {}
for name, gain, bstd in (('xavier', 1.0, 0.0), ('trained_like', 4.0, 0.1)):
    e = nicnes.Engine(max_batch=128, max_members=P, noise_len=1 << 27)
    try:
        S.setup_engine_workload(e, B=128, noise=noise, theta_gain=gain, bias_std=bstd)
        _, seq = e.evaluate(1, 0, P, 0.01, return_seq=True)
        seq = seq.cpu().numpy()                                   # [P, 2, B, T]
        T = seq.shape[-1]
        ended = seq == 0
        length = np.where(ended.any(-1), ended.argmax(-1) + 1, T)  # steps a row runs (its end token included)
        per_wg = length.reshape(P, -1).max(axis=1)                 # one 128-row slab per member at B = 128
        out[name] = {'mean_logit_steps_per_workgroup': float(per_wg.mean()), 'share_of_T': float(per_wg.mean() / T),
                     'workgroups_running_all_T': int((per_wg == T).sum()), 'mean_caption_length': float(length.mean())}
    finally:
        e.close()
print(json.dumps(out, indent=1))
