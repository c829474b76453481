"""The N>1 path of nicnes.population.PopulationRunner over gloo, world_size 2, on CPU: sharded
members + all-gather of fitness + all-reduce of the noise sum must give the same fitness and (to
fp32 summation-order rounding) the same theta as one rank evaluating everything."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tests.cpu_engine import OracleEngine, tiny_workload
from nicnes.population import PopulationRunner

P, ITERS, SIGMA = 4, 2, 0.02


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(rank, world, port, out_dir):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    if world > 1:
        dist.init_process_group('gloo', rank=rank, world_size=world)
    eng = OracleEngine(*tiny_workload())
    r = PopulationRunner(eng, P, SIGMA, l2coeff=1e-3, stepsize=1e-2, rank=rank, world_size=world)
    fits = []
    for it in range(1, ITERS + 1):
        f, ratio = r.step(it)
        fits.append(f.clone().numpy())
    np.savez(os.path.join(out_dir, 'r%d_w%d.npz' % (rank, world)), fits=np.stack(fits), theta=eng.theta32)
    if world > 1:
        dist.destroy_process_group()


def test_two_rank_gloo_matches_single_rank(tmp_path):
    _run(0, 1, _free_port(), str(tmp_path))
    mp.spawn(_run, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    one = np.load(tmp_path / 'r0_w1.npz')
    for rank in range(2):
        two = np.load(tmp_path / ('r%d_w2.npz' % rank))
        assert np.array_equal(one['fits'], two['fits'])
        assert np.allclose(one['theta'], two['theta'], rtol=0, atol=1e-6)
    # both ranks hold the identical replicated theta
    a, b = np.load(tmp_path / 'r0_w2.npz'), np.load(tmp_path / 'r1_w2.npz')
    assert np.array_equal(a['theta'], b['theta'])
