"""Ties bench.py's cpu_baseline (the restated reference worker, oracle/ref_worker.py) back to the true
reference: times the imported reference FCModel._sample (src/captioning/nets.py:183-245) and the
restatement on the same 640 rows (128 images x 5, as dataloader.py:175 duplicates them), one thread
each, as a worker pins (src/main.py:8-11). Runs in the build container only (imports /root/reference).

    PYTHONDONTWRITEBYTECODE=1 python scripts/time_port_vs_reference.py
"""
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'scripts'))
sys.path.insert(0, REPO)
import make_golden as G  # noqa: E402  (imports the reference modules)
from oracle import oracle as O  # noqa: E402
from oracle import ref_worker  # noqa: E402


def best_of(fn, n=3):
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        out = fn()
        ts.append(time.perf_counter() - t0)
    return min(ts), out


def main():
    torch.set_num_threads(1)
    torch.set_grad_enabled(False)
    d = O.Dims()
    theta = O.make_theta(d, 0, 1.0, 0.0)
    fc = np.repeat(np.random.Generator(np.random.PCG64(1234)).standard_normal((128, d.F)).astype(np.float32), 5, 0)
    fct = torch.from_numpy(fc)
    ref = G.ref_model(d)
    G.load_theta(ref, theta)
    ref.eval()
    port = ref_worker.FCModelRef()
    torch.nn.utils.vector_to_parameters(torch.from_numpy(theta), port.parameters())
    t_ref, (s_ref, _) = best_of(lambda: ref._sample(fct))
    t_port, (s_port, _) = best_of(lambda: port.sample(fct))
    print('reference FCModel._sample: %.3f s, restatement: %.3f s, ratio restatement/reference %.3f, tokens equal: %s'
          % (t_ref, t_port, t_port / t_ref, bool(torch.equal(s_ref, s_port))))


if __name__ == '__main__':
    main()
