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


def _run(rank, world, port, out_dir, chunks=4, pop=P):
    """chunks None: PopulationRunner's default exchange; every collective the iterations issue is counted"""
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    if world > 1:
        dist.init_process_group('gloo', rank=rank, world_size=world)
    calls = {'all_reduce': 0, 'all_gather_into_tensor': 0}

    def counted(name):
        f = getattr(dist, name)

        def g(*a, **k):
            calls[name] += 1
            return f(*a, **k)
        return g
    real = {n: getattr(dist, n) for n in calls}
    for n in calls:
        setattr(dist, n, counted(n))
    try:
        eng = OracleEngine(*tiny_workload())
        kw = {} if chunks is None else {'overlap_chunks': chunks}
        r = PopulationRunner(eng, pop, SIGMA, l2coeff=1e-3, stepsize=1e-2, rank=rank, world_size=world, **kw)
        if world > 1 and chunks is not None:
            assert len(r.ranges) == min(chunks, len(r.ranges)) and r.ranges[0][0] == 0 and r.ranges[-1][1] == eng.D
        fits = []
        for it in range(1, ITERS + 1):
            f, ratio = r.step(it)
            fits.append(f.clone().numpy())
    finally:
        for n, f in real.items():
            setattr(dist, n, f)
    np.savez(os.path.join(out_dir, 'r%d_w%d_c%s%s.npz' % (rank, world, chunks, '' if pop == P else '_p%d' % pop)), fits=np.stack(fits), theta=eng.theta32,
             all_reduce=calls['all_reduce'], all_gather=calls['all_gather_into_tensor'])
    if world > 1:
        dist.destroy_process_group()


def test_two_rank_gloo_matches_single_rank(tmp_path):
    _run(0, 1, _free_port(), str(tmp_path))
    mp.spawn(_run, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    one = np.load(tmp_path / 'r0_w1_c4.npz')
    for rank in range(2):
        two = np.load(tmp_path / ('r%d_w2_c4.npz' % rank))
        assert np.array_equal(one['fits'], two['fits'])
        assert np.allclose(one['theta'], two['theta'], rtol=0, atol=1e-6)
    # both ranks hold the identical replicated theta
    a, b = np.load(tmp_path / 'r0_w2_c4.npz'), np.load(tmp_path / 'r1_w2_c4.npz')
    assert np.array_equal(a['theta'], b['theta'])


def test_default_exchange_is_one_all_gather_and_one_all_reduce(tmp_path):
    """north_star's exchange by default: per iteration one all-gather of the fitness and ONE all-reduce of the
    noise sum (the range overlap is opt-in), with the same result as the explicit one-chunk runner"""
    for chunks in (None, 1):
        mp.spawn(_run, args=(2, _free_port(), str(tmp_path), chunks), nprocs=2, join=True)
    for rank in range(2):
        d, one = np.load(tmp_path / ('r%d_w2_cNone.npz' % rank)), np.load(tmp_path / ('r%d_w2_c1.npz' % rank))
        assert int(d['all_reduce']) == ITERS and int(d['all_gather']) == ITERS
        assert np.array_equal(d['fits'], one['fits']) and np.array_equal(d['theta'], one['theta'])


def test_overlapped_range_all_reduce_equals_one_all_reduce(tmp_path):
    """The noise sum in parameter ranges, each all-reduced while the next is summed (overlap_chunks), gives
    the same theta as one sum and one all-reduce."""
    for chunks in (1, 3):
        mp.spawn(_run, args=(2, _free_port(), str(tmp_path), chunks), nprocs=2, join=True)
    for rank in range(2):
        a, b = np.load(tmp_path / ('r%d_w2_c1.npz' % rank)), np.load(tmp_path / ('r%d_w2_c3.npz' % rank))
        assert np.array_equal(a['fits'], b['fits']) and np.array_equal(a['theta'], b['theta'])


def test_eight_rank_gloo_matches_single_rank(tmp_path):
    """World size 8 (the driver's 8-GPU node, rehearsed on gloo): P = 16 members, two per
    rank. Per iteration each rank issues exactly one all-gather and one all-reduce; fitness equals the
    single-rank run's, theta agrees to 1e-6 (but for Adam-amplified rounding in at most
    2 coordinates) and is identical on every rank."""
    pop = 16
    _run(0, 1, _free_port(), str(tmp_path), None, pop)
    mp.spawn(_run, args=(8, _free_port(), str(tmp_path), None, pop), nprocs=8, join=True)
    one = np.load(tmp_path / 'r0_w1_cNone_p16.npz')
    thetas = []
    for rank in range(8):
        d = np.load(tmp_path / ('r%d_w8_cNone_p16.npz' % rank))
        assert int(d['all_reduce']) == ITERS and int(d['all_gather']) == ITERS
        assert np.array_equal(one['fits'], d['fits'])
        # 8 partial noise sums add in another order than one; Adam's m / sqrt(v) step turns that rounding of a
        # near-zero gradient coordinate into up to ~20 ulp of theta (1 coordinate of 1,924 here)
        diff = np.abs(one['theta'] - d['theta'])
        assert diff.max() <= 4e-6 and (diff > 1e-6).sum() <= 2
        thetas.append(d['theta'])
    assert all(np.array_equal(thetas[0], t) for t in thetas[1:])


def _run_master(rank, world, port, out_dir):
    """EngineMaster.run (the NESMaster.run_master loop, nic_nes_master.py:56-168) sharded over gloo
    ranks, with a noise / step-size schedule reached mid-run."""
    from nicnes import config as C
    from nicnes import master as M
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    if world > 1:
        dist.init_process_group('gloo', rank=rank, world_size=world)
    dims, theta, fc, gts, df, n, table = tiny_workload()
    eng = OracleEngine(dims, theta, fc, gts, df, n, table)
    exp = {'algorithm': 'nic_nes', 'nb_offspring': P,
           'config': {'noise_stdev': SIGMA, 'batch_size': 4, 'l2coeff': 1e-3, 'snapshot_freq': 0,
                      'schedule_start': 1, 'schedule_limit': 2, 'stdev_divisor': 2, 'stepsize_divisor': 2},
           'policy_options': {'net': 'fc_caption', 'fitness': 'greedy', 'model_options': {}},
           'optimizer_options': {'type': 'adam', 'args': {'stepsize': 1e-2}}}
    spec = C.ExperimentSpec(exp, vocab_size=63)
    m = M.EngineMaster(spec, eng, log_dir=os.path.join(out_dir, 'log%d' % rank), rank=rank, world_size=world)
    m.run([{'fc_feats': fc, 'gts': gts}] * 3, max_iterations=3)
    np.savez(os.path.join(out_dir, 'm%d_w%d.npz' % (rank, world)), theta=eng.theta32,
             scores=np.array([r['score_mean'] for r in m.stats]), sigma=np.array([r['noise_stdev'] for r in m.stats]),
             stepsize=np.float64(m.opt.stepsize))
    if world > 1:
        dist.destroy_process_group()


def test_two_rank_engine_master_run_matches_single_rank(tmp_path):
    _run_master(0, 1, _free_port(), str(tmp_path))
    mp.spawn(_run_master, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    one = np.load(tmp_path / 'm0_w1.npz')
    for rank in range(2):
        two = np.load(tmp_path / ('m%d_w2.npz' % rank))
        assert np.array_equal(one['scores'], two['scores']) and np.array_equal(one['sigma'], two['sigma'])
        assert float(two['stepsize']) == float(one['stepsize']) == 1e-2 / 4
        assert np.allclose(one['theta'], two['theta'], rtol=0, atol=1e-6)
    assert np.array_equal(np.load(tmp_path / 'm0_w2.npz')['theta'], np.load(tmp_path / 'm1_w2.npz')['theta'])
