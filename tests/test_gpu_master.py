"""The master loop on the HIP engine against the oracle engine (tests/cpu_engine.OracleEngine, the
CPU restatement of every kernel), and the engine's C-ABI RCCL collectives.

* EngineMaster.run (NESMaster.run_master, nic_nes_master.py:56-168) for 3 iterations with a
  noise / batch-size / step-size schedule reached after iteration 1 (tools/iteration.py:149-187):
  the batch grows from 8 to 16 images past the size the engine was created with, so the engine's
  batch buffers are re-created; per-iteration fitness to 1e-9 relative, theta / m / v to 1e-6.
* nicnes_comm_init + nicnes_allgather_fitness + nicnes_allreduce_grad at one rank (the only
  RCCL shape a one-GPU box can run): identity exchanges, then one PopulationRunner step on
  comm='engine' equals the torch.distributed-free single-rank step bit for bit."""
import numpy as np
import pytest

torch = pytest.importorskip('torch')

pytestmark = pytest.mark.gpu

from oracle import oracle as O          # noqa: E402
from tests.cpu_engine import OracleEngine  # noqa: E402

NOISE_LEN = 1 << 23


class _Loader:
    def __init__(self, fc, gts):
        self.fc, self.gts, self.pos, self.sizes = fc, gts, 0, []

    def get_batch(self, split, batch_size=None):
        self.sizes.append(batch_size)
        ix = [(self.pos + k) % len(self.gts) for k in range(batch_size)]
        self.pos += batch_size
        return {'fc_feats': np.repeat(self.fc[ix], 5, axis=0), 'gts': [self.gts[i] for i in ix]}


def _spec(P):
    from nicnes import config as C
    exp = {'algorithm': 'nic_nes', 'nb_offspring': P,
           'config': {'noise_stdev': 0.01, 'batch_size': 8, 'l2coeff': 1e-3, 'snapshot_freq': 0, 'single_batch': True,
                      'schedule_start': 1, 'schedule_limit': 2, 'bs_multiplier': 2, 'stdev_divisor': 2,
                      'stepsize_divisor': 2},
           'policy_options': {'net': 'fc_caption', 'fitness': 'greedy', 'model_options': {}},
           'optimizer_options': {'type': 'adam', 'args': {'stepsize': 1e-3}}}
    return C.ExperimentSpec(exp)


def test_master_trajectory_with_batch_growth_matches_oracle_engine():
    import nicnes
    import nicnes.synthetic as S
    from nicnes import master as M
    dims = O.Dims()
    theta = O.make_theta(dims, 0, 4.0, 0.1)
    fc = np.random.Generator(np.random.PCG64(1234)).standard_normal((16, dims.F)).astype(np.float32)
    base, _, _ = O.decode(dims, theta, fc)
    gts, df, n = S.build_references(base, dims.vocab_size, seed=9, n_refs=5, df_sets=128)
    table = O.noise_table(NOISE_LEN, 123)
    P = 4
    e = nicnes.Engine(max_batch=8, max_members=P, noise_len=NOISE_LEN, noise_seed=0)
    try:
        e.set_noise_table(table)
        keys, vals = nicnes.df_table_arrays(df)
        e.set_df_table(keys, vals, np.log(float(n)))
        gpu = M.EngineMaster(_spec(P), e, theta=theta)
        ora_e = OracleEngine(dims, theta, fc, gts, df, n, table, noise_seed=0)
        ora = M.EngineMaster(_spec(P), ora_e, theta=theta)
        la, lb = _Loader(fc, gts), _Loader(fc, gts)
        gpu.run(la, max_iterations=3)
        ora.run(lb, max_iterations=3)
        assert la.sizes == lb.sizes == [8, 16, 16]
        assert e.cfg.max_batch == 8           # the Python config is the creation size; the handle grew
        for a, b in zip(gpu.stats, ora.stats):
            for k in ('score_mean', 'score_max', 'score_min'):
                assert abs(a[k] - b[k]) <= 1e-9 * max(1.0, abs(b[k])), (k, a[k], b[k])
            assert a['batch_size'] == b['batch_size'] and a['noise_stdev'] == b['noise_stdev']
        t64 = e.theta()[0].cpu().numpy()
        assert np.allclose(t64, ora_e.adam.theta, rtol=1e-6, atol=1e-12)
        m, v, t = e.adam_state()
        assert t == 3 and np.allclose(m.cpu().numpy(), ora_e.adam.m, rtol=1e-6, atol=1e-15)
        assert np.allclose(v.cpu().numpy(), ora_e.adam.v, rtol=1e-6, atol=1e-20)
        assert gpu.opt.stepsize == ora.opt.stepsize == 1e-3 / 4      # reached at iterations 1 and 3
    finally:
        e.close()


def test_engine_rccl_collectives_single_rank():
    import nicnes
    import nicnes.synthetic as S
    from nicnes.population import PopulationRunner
    P = 4
    e = nicnes.Engine(max_batch=16, max_members=P, noise_len=NOISE_LEN, noise_seed=3)
    try:
        S.setup_engine_workload(e, B=16, noise=O.noise_table(NOISE_LEN, 123), df_sets=64)
        uid = nicnes.Engine.comm_unique_id()
        assert len(uid) == 128
        e.comm_init(1, 0, uid)
        fl = torch.arange(2 * P, dtype=torch.float64, device=e.device).reshape(P, 2)
        fa = torch.empty_like(fl)
        e.allgather_fitness(fl, fa)
        g = torch.linspace(-1, 1, e.D, dtype=torch.float32, device=e.device)
        g0 = g.clone()
        e.allreduce_grad(g)
        torch.cuda.synchronize()
        assert torch.equal(fa, fl) and torch.equal(g, g0)
        th0 = e.theta()[0].clone()
        r1 = PopulationRunner(e, P, 0.01, l2coeff=1e-7, stepsize=1e-3, comm='engine')
        f1, _ = r1.step(1)
        t1 = e.theta()[0].clone()
        e.set_theta(th0.float().cpu().numpy())          # fp32 origin again (first-step semantics)
        e.set_adam_state(np.zeros(e.D), np.zeros(e.D), 0)
        r0 = PopulationRunner(e, P, 0.01, l2coeff=1e-7, stepsize=1e-3)
        f0, _ = r0.step(1)
        assert torch.equal(f0, f1) and torch.equal(e.theta()[0], t1)
        e.comm_destroy()
    finally:
        e.close()
