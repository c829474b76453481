"""GPU: nicnes_evaluate_theta, the eval rollout of theta itself (CaptPolicy.rollout,
/root/reference/src/captioning/policies.py:86-128, run for the eval result of
nic_nes_worker.py:65-70) decoded ONCE, sign + over the first half of the images and sign - over the
rest. At sigma = 0 both signs are theta, so the result must equal the sign-+ row of a sigma = 0
member of nicnes_evaluate_lp (which decodes the whole batch twice): tokens and greedy fitness bit for
bit, log-probs to 2 ulp (the decode shape may differ), on every decode path, for even and odd batch sizes, batches spanning several slabs, the
greedy_* criteria and per-member batches; and the fitness equals the oracle's."""
import numpy as np
import pytest

torch = pytest.importorskip('torch')

pytestmark = pytest.mark.gpu

from oracle import oracle as O          # noqa: E402
from oracle import cider_ref as CR      # noqa: E402

NOISE_LEN = 1 << 23


@pytest.fixture(scope='module')
def eng():
    import nicnes
    assert torch.cuda.is_available(), 'GPU tests need a GPU'
    e = nicnes.Engine(max_batch=300, max_members=4, noise_len=NOISE_LEN, noise_seed=7)
    e.set_noise_table(O.noise_table(NOISE_LEN, 123))
    yield e
    e.close()


def _batch(dims, theta, B, seed):
    import nicnes.synthetic as S
    fc = np.random.Generator(np.random.PCG64(seed)).standard_normal((B, dims.F)).astype(np.float32)
    base, _, _ = O.decode(dims, theta, fc)
    gts, df, n = S.build_references(base, dims.vocab_size, seed=seed + 1, df_sets=64)
    return fc, gts, df, n


def _load(eng, theta, batches, df, n):
    import nicnes
    eng.set_theta(theta)
    keys, vals = nicnes.df_table_arrays(df)
    eng.set_df_table(keys, vals, np.log(float(n)))
    eng.set_batches([(fc, gts) for fc, gts in batches])


PATHS = {'auto': (0, 0, 1), 'fused': (1, 4, 1), 'fused64': (1, 2, 1), 'coop': (4, 4, 1), 'split': (4, 4, 0)}


@pytest.mark.parametrize('B', [40, 41, 128, 257])
@pytest.mark.parametrize('path', list(PATHS))
def test_eval_theta_equals_the_sigma0_member(eng, B, path):
    dims = O.Dims()
    theta = O.make_theta(dims, 2, 4.0, 0.1)
    fc, gts, df, n = _batch(dims, theta, B, 100 + B)
    _load(eng, theta, [(fc, gts)], df, n)
    S, G, coop = PATHS[path]
    try:
        eng.set_decode_split(S, G)
        eng.set_decode_coop(coop)
        for mode in ('greedy', 'greedy_linprob'):
            eng.set_fitness_mode(mode)
            f2, seq2, lp2 = eng.evaluate(0, 0, 1, 0.0, return_seq=True, return_lp=True)
            f1, seq1, lp1 = eng.evaluate_theta(0, return_seq=True, return_lp=True)
            f0 = eng.evaluate_theta(0)
            f2, f1, f0 = f2.cpu().numpy(), f1.cpu().numpy(), f0.cpu().numpy()
            # tokens bit-exact; the log-probs to 2 ulp: half the rows per sign can change the decode shape
            # (vocabulary ranges S), which merges the row's exp-sum in another order (lse's last bit)
            assert np.array_equal(seq1.cpu().numpy(), seq2[0, 0].cpu().numpy()), mode
            np.testing.assert_allclose(lp1.cpu().numpy(), lp2[0, 0].cpu().numpy(), rtol=2.5e-7, atol=0)
            assert f2[0, 0] == f2[0, 1] and f0[0] == f1[0], (mode, f1, f2, f0)
            if mode == 'greedy':
                assert f1[0] == f2[0, 0], (f1, f2)
            else:
                assert abs(f1[0] - f2[0, 0]) <= 1e-6 * abs(f2[0, 0]), (f1, f2)
            if mode == 'greedy':
                oseq, olp, fr = O.decode(dims, theta, fc)
                f_ref, _ = CR.rollout_fitness(CR.CiderDOracle(df, n), oseq, gts)
                if not fr.any():
                    assert np.array_equal(seq1.cpu().numpy(), oseq)
                    assert abs(f1[0] - f_ref) <= 1e-9 * max(1.0, abs(f_ref))
    finally:
        eng.set_fitness_mode('greedy')
        eng.set_decode_split(0, 0)
        eng.set_decode_coop(1)


def test_eval_theta_on_a_named_batch(eng):
    """set_batches with three batches: evaluate_theta(b) scores batch b (member_batch of a sigma = 0 member)."""
    dims = O.Dims()
    theta = O.make_theta(dims, 3, 4.0, 0.1)
    batches, df_all, n = [], {}, 0
    for j in range(3):
        fc, gts, df, n = _batch(dims, theta, 33, 7 * j + 1)
        batches.append((fc, gts))
        df_all = df
    _load(eng, theta, batches, df_all, n)
    for b in range(3):
        f2 = eng.evaluate(0, 0, 1, 0.0, member_batch=[b]).cpu().numpy()
        f1 = eng.evaluate_theta(b).cpu().numpy()
        assert f1[0] == f2[0, 0], (b, f1, f2)
    with pytest.raises(Exception):
        eng.evaluate_theta(3)


def test_eval_theta_sampled_draws_follow_the_iteration(eng):
    """Sampled modes: an eval rollout draws from its own stream per iteration, reproducibly, and not
    from an evolve member's (the sigma = 0 member 0 of the same iteration decodes other captions)."""
    dims = O.Dims()
    theta = O.make_theta(dims, 2, 4.0, 0.1)
    fc, gts, df, n = _batch(dims, theta, 40, 7)
    _load(eng, theta, [(fc, gts)], df, n)
    try:
        eng.set_fitness_mode('sample')
        _, s1 = eng.evaluate_theta(0, return_seq=True, iteration=1)
        _, s1b = eng.evaluate_theta(0, return_seq=True, iteration=1)
        _, s2 = eng.evaluate_theta(0, return_seq=True, iteration=2)
        _, sm = eng.evaluate(1, 0, 1, 0.0, return_seq=True)
        assert torch.equal(s1, s1b)
        assert not torch.equal(s1, s2)
        assert not torch.equal(s1, sm[0, 0])
    finally:
        eng.set_fitness_mode('greedy')
