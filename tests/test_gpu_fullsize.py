"""The bench configuration itself (BASELINE.json configs[2]: fc_caption, P = 512 antithetic members,
B = 128 unique images, sigma 0.01, the 2^27 shared table) checked end to end on the GPU:
  * 16 members spread over the population: greedy tokens bit-exact vs the oracle decode (except
    after an lse-fragile step), CIDEr-D fitness to 1e-9 vs the oracle scorer;
  * shard invariance: the population evaluated as [0, 200) + [200, 512) equals one launch bit for bit;
  * centred ranks and weights bit-exact vs the restatement of compute_centered_ranks;
  * the weighted noise sum bit-exact vs its fp64 restatement on 4096 sampled coordinates;
  * one Adam step through PopulationRunner (the bench's step) with a finite ratio, and theta moved
    by exactly the engine's own step.
"""
import numpy as np
import pytest

torch = pytest.importorskip('torch')

pytestmark = pytest.mark.gpu

from oracle import oracle as O          # noqa: E402
from oracle import cider_ref as CR      # noqa: E402

P, B, SIGMA, T_LEN, IT = 512, 128, 0.01, 1 << 27, 1


@pytest.fixture(scope='module')
def full():
    import nicnes
    import nicnes.synthetic as S
    assert torch.cuda.is_available(), 'GPU tests need a GPU'
    e = nicnes.Engine(max_batch=B, max_members=P, noise_len=T_LEN, noise_seed=0)
    table = O.noise_table(T_LEN, 123)
    wl = S.setup_engine_workload(e, B=B, noise=table)
    yield e, table, wl
    e.close()


def test_bench_config_tokens_and_fitness(full):
    e, table, wl = full
    dims = O.Dims()
    fit, seq = e.evaluate(IT, 0, P, SIGMA, return_seq=True)
    fit, seq = fit.cpu().numpy(), seq.cpu().numpy()
    idx = e.noise_indices(IT, 0, P).cpu().numpy()
    scorer = CR.CiderDOracle(wl['df'], wl['ref_len_raw'])
    for i in np.linspace(0, P - 1, 16).astype(int):
        assert idx[i] == O.noise_index(0, IT, int(i), T_LEN, dims.D)
        for s, sign in enumerate((+1, -1)):
            oseq, _, fr = O.decode(dims, O.perturb(wl['theta32'], table, int(idx[i]), SIGMA, sign), wl['fc'])
            for b in range(B):
                for t in range(dims.T):
                    if fr[b, t]:
                        break
                    assert seq[i, s, b, t] == oseq[b, t], (i, s, b, t)
            f_ref, _ = CR.rollout_fitness(scorer, seq[i, s], wl['gts'])
            assert abs(fit[i, s] - f_ref) <= 1e-9 * max(1.0, f_ref), (i, s, fit[i, s], f_ref)
    assert np.isfinite(fit).all() and fit.std() > 0


def test_bench_config_shards_ranks_noise_sum(full):
    e, table, wl = full
    dims = O.Dims()
    f_all = e.evaluate(IT, 0, P, SIGMA).clone()
    f_a = e.evaluate(IT, 0, 200, SIGMA).clone()
    f_b = e.evaluate(IT, 200, P - 200, SIGMA).clone()
    assert torch.equal(torch.cat([f_a, f_b]), f_all)
    cr, w = e.rank_weights(f_all)
    w_ref, cr_ref = O.weights_from_fitness(f_all.cpu().numpy())
    assert np.array_equal(cr.cpu().numpy(), cr_ref) and np.array_equal(w.cpu().numpy(), w_ref)
    g = e.grad_partial(IT, 0, P, w, SIGMA).cpu().numpy()
    idx = e.noise_indices(IT, 0, P).cpu().numpy().astype(np.int64)
    J = np.sort(np.random.default_rng(3).choice(dims.D, 4096, replace=False))
    acc = np.zeros(J.size, np.float64)
    for i in range(P):
        acc += np.float64(w_ref[i]) * (np.float32(SIGMA) * table[idx[i] + J]).astype(np.float64)
    assert np.array_equal(g[J], acc.astype(np.float32))


def test_bench_config_runner_step(full):
    e, table, wl = full
    from nicnes.population import PopulationRunner
    th0 = e.theta()[0].cpu().numpy()
    r = PopulationRunner(e, P, SIGMA, l2coeff=1e-7, stepsize=1e-3)
    fit_all, ratio = r.step(IT + 1)
    th1, th32 = (t.cpu() for t in e.theta())
    ratio = float(ratio)
    assert np.isfinite(ratio) and ratio > 0
    step = th1.numpy() - th0
    assert np.isclose(np.linalg.norm(step) / np.linalg.norm(th0), ratio, rtol=1e-9)
    assert torch.equal(th32, th1.float())
