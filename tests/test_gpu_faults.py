"""GPU: a decode that loses rows is contained inside its own iteration.

Two device-side spins are bounded: a coop workgroup waiting for its group's partners
(nicnes_decode_coop_kernel, 0.5 s) and a sampled workgroup looking for a free logit slot. When either
gives up, rows stay undecoded. The same iteration must not consume them: the CIDEr-D epilogue writes
NaN fitness, the noise sum comes back NaN (so an all-reduce carries the fault to every rank), and the
optimizer step is a device-side no-op (theta, m, v unchanged), all without a host wait. The error is
raised at the next host read (the next evaluate, or the update ratio). Test hooks force each spin past
its bound: NICNES_TEST_COOP_STALL (ms) starts coop workgroup 0 late; NICNES_TEST_SLOTS gives the
sampled decode fewer logit slots than it has workgroups.

Also here: the coop grid is bounded by the occupancy query (the split path takes larger grids),
and nicnes_evaluate_theta writes exactly its rows_total x T outputs at odd batch sizes."""
import ctypes
import os

import numpy as np
import pytest

torch = pytest.importorskip('torch')

pytestmark = pytest.mark.gpu

from oracle import oracle as O          # noqa: E402

NOISE_LEN = 1 << 23
SIGMA = 0.01


def _engine(max_batch=128, max_members=8, seed=11):
    import nicnes
    assert torch.cuda.is_available(), 'GPU tests need a GPU'
    e = nicnes.Engine(max_batch=max_batch, max_members=max_members, noise_len=NOISE_LEN, noise_seed=seed)
    e.set_noise_table(O.noise_table(NOISE_LEN, 123))
    return e


def _load(e, B, seed=3):
    import nicnes
    dims = O.Dims()
    e.set_theta(O.make_theta(dims, seed, 4.0, 0.1))
    fc = np.random.Generator(np.random.PCG64(seed)).standard_normal((B, 2048)).astype(np.float32)
    gts = [np.asarray([[(7 * b + k) % 60 + 1 for k in range(8)] + [0] * 8], np.int32) for b in range(B)]
    keys, vals = nicnes.df_table_arrays({})
    e.set_df_table(keys, vals, np.log(4096.0))
    e.set_batch(fc, gts)


def _iteration(e, P):
    """evaluate -> ranks -> noise sum -> Adam, enqueued without a host wait (PopulationRunner.step order)"""
    fit = e.evaluate(1, 0, P, SIGMA)
    _, w = e.rank_weights(fit)
    gsum = e.grad_partial(1, 0, P, w, SIGMA)
    e.adam_step(gsum, P, 0.005, 0.01, sync=False)
    return fit, gsum


def _contained(e, P, counter):
    from nicnes import NicnesError
    th0, m0, v0 = e.theta()[0].clone(), *[x.clone() for x in e.adam_state()[:2]]
    fit, gsum = _iteration(e, P)
    torch.cuda.synchronize()
    assert e.stats()[counter] > 0
    assert torch.isnan(fit).all(), fit
    assert torch.isnan(gsum).all()
    th1, (m1, v1, _) = e.theta()[0], e.adam_state()
    assert torch.equal(th0, th1) and torch.equal(m0, m1) and torch.equal(v0, v1)
    with pytest.raises(NicnesError):
        e.last_ratio()
    with pytest.raises(NicnesError):
        e.evaluate(2, 0, P, SIGMA)


def test_coop_partner_timeout_is_contained(monkeypatch):
    monkeypatch.setenv('NICNES_TEST_COOP_STALL', '700')      # past the 0.5 s spin bound
    e = _engine()
    try:
        _load(e, 128)
        e.set_decode_split(4, 4)
        assert e.decode_path(128, 4) == 'coop'
        _contained(e, 4, 'coop_timeouts')
    finally:
        e.close()


def test_sampled_slot_timeout_is_contained(monkeypatch):
    monkeypatch.setenv('NICNES_TEST_SLOTS', '1')             # 8 workgroups of ~0.2 s share one slot
    e = _engine(max_batch=640)
    try:
        e.set_fitness_mode('sample')
        e.set_rows_per_image(5)
        _load(e, 128)
        _contained(e, 8, 'sample_slot_timeouts')
    finally:
        e.close()


def test_faulted_rank_poisons_the_reduced_sum():
    """another rank's poisoned noise sum (NaN everywhere after the all-reduce): this rank's Adam step is a
    no-op too and the ratio read raises"""
    from nicnes import NicnesError
    e = _engine()
    try:
        _load(e, 128)
        th0 = e.theta()[0].clone()
        gsum = torch.full((e.D,), float('nan'), dtype=torch.float32, device=e.device)
        with pytest.raises(NicnesError):
            e.adam_step(gsum, 4, 0.005, 0.01)
        assert torch.equal(th0, e.theta()[0])
        # a healthy handle: a finite sum steps as before
        gsum.zero_()
        e.adam_step(gsum, 4, 0.005, 0.01)
    finally:
        e.close()


def test_healthy_iterations_unaffected():
    """no hook: the coop and fused iterations run, fitness finite, no counters move"""
    e = _engine(max_members=64)
    try:
        _load(e, 128)
        for split in ((4, 4), (0, 0)):
            e.set_decode_split(*split)
            fit, gsum = _iteration(e, 8)
            assert torch.isfinite(fit).all() and torch.isfinite(gsum).all()
            assert np.isfinite(e.last_ratio())
        s = e.stats()
        assert s['coop_timeouts'] == 0 and s['sample_slot_timeouts'] == 0
    finally:
        e.close()


def test_coop_grid_bounded_by_residency():
    """the coop path takes a grid only while every workgroup can be resident at once (occupancy x CUs); one
    member slab more at S = 4 goes to the two-launch split path, with the same tokens"""
    e = _engine(max_members=512)
    try:
        _load(e, 128)
        e.set_decode_split(4, 4)
        P = e.n_cu // 4
        assert e.decode_path(128, P) == 'coop' and e.decode_path(128, P + 1) == 'split'
        fit, seq = e.evaluate(1, 0, P + 1, SIGMA, return_seq=True)
        fit_c, seq_c = e.evaluate(1, 0, P, SIGMA, return_seq=True)
        assert torch.equal(seq[:P], seq_c) and torch.equal(fit[:P], fit_c)
    finally:
        e.close()


@pytest.mark.parametrize('B', [41, 257])
def test_eval_theta_writes_exactly_its_rows(B):
    """odd B: sign + decodes ceil(B/2) images, sign - the rest; the caller's [B, T] buffers are written and
    not one element past them (canaries after an exact-size view)"""
    from nicnes import _lib
    e = _engine(max_batch=300, max_members=2)
    try:
        _load(e, B, seed=9)
        e.set_fitness_mode('greedy_linprob')                  # writes log-probs too
        T = e.cfg.seq_length
        seq = torch.full((B + 2, T), -7, dtype=torch.int32, device=e.device)
        lp = torch.full((B + 2, T), -7.0, dtype=torch.float32, device=e.device)
        fit = torch.empty(1, dtype=torch.float64, device=e.device)
        with torch.cuda.device(e.device):
            _lib.check(e.L.nicnes_evaluate_theta(e.h, 0, 0, ctypes.c_void_p(fit.data_ptr()),
                                                 ctypes.c_void_p(seq.data_ptr()), ctypes.c_void_p(lp.data_ptr()),
                                                 e._stream()), e.h, 'evaluate_theta')
        torch.cuda.synchronize()
        assert (seq[B:] == -7).all() and (lp[B:] == -7.0).all()
        ref_fit, ref_seq, ref_lp = e.evaluate_theta(0, return_seq=True, return_lp=True)
        assert torch.equal(seq[:B], ref_seq) and torch.equal(lp[:B], ref_lp) and torch.equal(fit, ref_fit)
    finally:
        e.close()


def _master_spec(P):
    from nicnes import config as C
    exp = {'algorithm': 'nic_nes', 'nb_offspring': P,
           'config': {'noise_stdev': 0.01, 'batch_size': 128, 'l2coeff': 1e-3, 'snapshot_freq': 0, 'single_batch': True},
           'policy_options': {'net': 'fc_caption', 'fitness': 'greedy', 'model_options': {}},
           'optimizer_options': {'type': 'adam', 'args': {'stepsize': 1e-2}}}
    return C.ExperimentSpec(exp)


def _master_run(monkeypatch, tmp_path, stall_launches, iterations=2, retries=1):
    """EngineMaster.run on the coop path (P = 4 members, S = 4) with the first `stall_launches` coop launches
    stalled past the spin bound (0: no fault). Returns (master, engine); the caller closes the engine."""
    import nicnes
    from nicnes import master as M
    if stall_launches:
        monkeypatch.setenv('NICNES_TEST_COOP_STALL', '700')
        monkeypatch.setenv('NICNES_TEST_COOP_STALL_LAUNCHES', str(stall_launches))
    e = _engine()
    monkeypatch.delenv('NICNES_TEST_COOP_STALL', raising=False)
    monkeypatch.delenv('NICNES_TEST_COOP_STALL_LAUNCHES', raising=False)
    _load(e, 128)
    e.set_decode_split(4, 4)
    assert e.decode_path(128, 4) == 'coop'
    fc = np.random.Generator(np.random.PCG64(3)).standard_normal((128, 2048)).astype(np.float32)
    gts = [np.asarray([[(7 * b + k) % 60 + 1 for k in range(8)] + [0] * 8], np.int32) for b in range(128)]
    m = M.EngineMaster(_master_spec(4), e, log_dir=str(tmp_path), theta=e.theta()[1].cpu().numpy())
    try:
        m.run([(fc, gts)] * iterations, max_iterations=iterations, fault_retries=retries)
    except Exception:
        e.close()
        raise
    return m, e


def test_master_reruns_a_faulted_iteration(monkeypatch, tmp_path):
    """one coop hand-off timeout in iteration 1 is recorded, the handle's fault cleared and the
    iteration re-run; the run then ends exactly as an unfaulted run (theta, m, v, t, fitness bit for bit)."""
    import json
    import os
    ref, e0 = _master_run(monkeypatch, tmp_path / 'clean', 0)
    try:
        got, e1 = _master_run(monkeypatch, tmp_path / 'faulted', 1)
        try:
            assert ref.faults == [] and len(got.faults) == 1
            f = got.faults[0]
            assert f['iter'] == 1 and f['attempt'] == 0 and f['coop_timeouts'] > 0 and 'hand-off' in f['error']
            assert os.path.exists(tmp_path / 'faulted' / 'faults' / 'fault_i1_a0.json')
            with open(tmp_path / 'faulted' / 'faults' / 'fault_i1_a0.json') as fh:
                assert json.load(fh)['iter'] == 1
            assert [s['score_mean'] for s in got.stats] == [s['score_mean'] for s in ref.stats]
            assert [s['update_ratio'] for s in got.stats] == [s['update_ratio'] for s in ref.stats]
            for a, b in zip(e1.adam_state()[:2] + e1.theta(), e0.adam_state()[:2] + e0.theta()):
                assert torch.equal(a, b)
            assert e1.adam_state()[2] == e0.adam_state()[2] == 2
            assert e1.stats()['coop_timeouts'] == 0                 # cleared
        finally:
            e1.close()
    finally:
        e0.close()


def test_master_gives_up_after_the_retries_with_a_snapshot(monkeypatch, tmp_path):
    """Two faulted tries of iteration 1 with fault_retries=1: DecodeFault propagates (the process would exit
    non-zero), both tries are recorded, theta / m / v / t are the initial ones and a resumable snapshot exists."""
    import glob
    import nicnes
    with pytest.raises(nicnes.DecodeFault):
        _master_run(monkeypatch, tmp_path, 2, iterations=1, retries=1)
    assert sorted(os.path.basename(p) for p in glob.glob(str(tmp_path / 'faults' / '*.json'))) == \
        ['fault_i1_a0.json', 'fault_i1_a1.json']
    assert glob.glob(str(tmp_path / 'snapshot' / 'z_info_e*_i0-0.json'))    # the pre-fault state: iteration 0
    assert os.path.exists(tmp_path / 'snapshot' / 'optimizer.tar')
    from nicnes import nes as N
    st = N._load_state(str(tmp_path / 'snapshot' / 'optimizer.tar'))
    assert st['t'] == 0 and not np.any(st['m'])
