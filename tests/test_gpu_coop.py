"""GPU parity of the coop decode path (nicnes_decode_coop_kernel): the split shape (128-row slabs,
S = 2 or 4 logit ranges per member slab) in ONE persistent launch whose workgroups hand the partial
greedy states and h' to each other inside it. This is the shape of 64 and 128 members per GPU at
B = 128: configs[1], and the metric's pop=512 over 8 and 4 GPUs.

Bars: tokens and log-probs bit-identical to the two-launch split path (same merge order of the
partials), tokens equal to the C oracle except after a step it marks lse-fragile, CIDEr-D fitness to
1e-9 relative, no hand-off timeout; two-slab batches (B = 130), the early exit, the forced exact pass
and the bounded-lse undecided rows included."""
import numpy as np
import pytest

torch = pytest.importorskip('torch')

pytestmark = pytest.mark.gpu

from oracle import oracle as O          # noqa: E402
from oracle import cider_ref as CR      # noqa: E402

NOISE_LEN = 1 << 23
SIGMA = 0.01


def _fc(B, seed):
    return np.random.Generator(np.random.PCG64(seed)).standard_normal((B, 2048)).astype(np.float32)


def _engine(max_batch=130, max_members=128, seed=5):
    import nicnes
    assert torch.cuda.is_available(), 'GPU tests need a GPU'
    e = nicnes.Engine(max_batch=max_batch, max_members=max_members, noise_len=NOISE_LEN, noise_seed=seed)
    e._table_np = O.noise_table(NOISE_LEN, 123)
    e.set_noise_table(e._table_np)
    return e


def _load(e, theta, fc, gts=None, df=None, n=4096):
    import nicnes
    e.set_theta(theta)
    if gts is None:
        gts = [np.asarray([[(7 * b + k) % 60 + 1 for k in range(8)] + [0] * 8], np.int32) for b in range(fc.shape[0])]
    keys, vals = nicnes.df_table_arrays(df or {})
    e.set_df_table(keys, vals, np.log(float(n)))
    e.set_batch(fc, gts)
    return gts


def _mismatch(gpu, ora, fragile):
    bad = []
    for b in range(ora.shape[0]):
        for t in range(ora.shape[1]):
            if fragile[b, t]:
                break
            if gpu[b, t] != ora[b, t]:
                bad.append((b, t))
                break
    return bad


@pytest.fixture(scope='module')
def eng():
    e = _engine()
    yield e
    assert e.stats()['coop_timeouts'] == 0
    e.close()


def test_decode_path_rule(eng):
    """the coop path takes exactly the split shapes whose workgroups all fit on the GPU at once"""
    if eng.n_cu != 256:
        pytest.skip('shape rule checked on the 256-CU MI355X')
    assert eng.decode_path(128, 64) == 'coop' and eng.decode_shape(128, 64) == (4, 1, 4)
    assert eng.decode_path(128, 128) == 'coop' and eng.decode_shape(128, 128) == (4, 1, 2)
    assert eng.decode_path(128, 256) == 'fused' and eng.decode_path(128, 512) == 'fused'
    assert eng.decode_path(64, 64) == 'split'                  # 64-row slabs stay on the two-launch path ...
    assert eng.decode_path(64, 512) == 'fused' and eng.decode_shape(64, 512) == (2, 1, 1)   # ... unless S = 1
    assert eng.decode_path(130, 64) == 'split'                 # B = 130 pads least with 64-row slabs
    eng.set_decode_split(0, 4)                                # forced 128-row slabs: two of them
    try:
        assert eng.decode_path(130, 64) == 'coop' and eng.decode_shape(130, 64) == (4, 2, 2)
        eng.set_decode_coop(0)
        assert eng.decode_path(128, 64) == 'split'
    finally:
        eng.set_decode_coop(1)
        eng.set_decode_split(0, 0)


@pytest.mark.parametrize('B,P', [(128, 64), (128, 128), (130, 64), (100, 3)],
                         ids=['pop64_S4', 'pop128_S2', 'two_slabs_S2', 'ragged_3members'])
def test_coop_equals_split_and_oracle(eng, B, P):
    dims = O.Dims()
    theta = O.make_theta(dims, 6, 4.0, 0.1)
    fc = _fc(B, 321 + B)
    _load(eng, theta, fc)
    if P < 8:
        eng.set_decode_split(4, 4)                # a few members: the automatic rule would split wider
    elif B > 128:
        eng.set_decode_split(0, 4)                # two 128-row slabs (the automatic rule takes 64-row ones)
    try:
        assert eng.decode_path(B, P) == 'coop'
        fit_c, seq_c, lp_c = eng.evaluate(4, 5, P, SIGMA, return_seq=True, return_lp=True)
        eng.set_decode_coop(0)
        assert eng.decode_path(B, P) == 'split'
        fit_s, seq_s, lp_s = eng.evaluate(4, 5, P, SIGMA, return_seq=True, return_lp=True)
    finally:
        eng.set_decode_coop(1)
        eng.set_decode_split(0, 0)
    assert torch.equal(seq_c, seq_s) and torch.equal(lp_c, lp_s) and torch.equal(fit_c, fit_s)
    seq = seq_c.cpu().numpy()
    idx = eng.noise_indices(4, 5, P).cpu().numpy()
    for k in sorted({0, P // 2, P - 1}):
        for s, sign in enumerate((+1, -1)):
            oseq, _, fr = O.decode(dims, O.perturb(theta, eng._table_np, int(idx[k]), SIGMA, sign), fc)
            assert _mismatch(seq[k, s], oseq, fr) == [], (k, s)


def test_coop_bench_workload_fitness(eng):
    """xavier theta and references from its own base caption (the bench workload): fitness equal to the
    restated CIDEr-D of the coop tokens, and greedy-only (bounded lse) tokens equal to the exact-sum ones"""
    import nicnes.synthetic as S
    dims = O.Dims()
    theta = S.init_theta(S.Dims(), 0)
    fc = _fc(128, 1234)
    base, _, _ = O.decode(dims, theta, fc)
    gts, df, n = S.build_references(base, dims.vocab_size, seed=4321, n_refs=5, df_sets=512)
    _load(eng, theta, fc, gts, df, n)
    fit, seq = eng.evaluate(1, 0, 64, SIGMA, return_seq=True)           # greedy-only: bounded lse
    _, seq_lp, _ = eng.evaluate(1, 0, 64, SIGMA, return_seq=True, return_lp=True)   # exact exp-sum
    assert torch.equal(seq, seq_lp)
    fit, seq = fit.cpu().numpy(), seq.cpu().numpy()
    scorer = CR.CiderDOracle(df, n)
    for i in (0, 17, 63):
        for s in range(2):
            f_ref, _ = CR.rollout_fitness(scorer, seq[i, s], gts)
            assert abs(fit[i, s] - f_ref) <= 1e-9 * max(1.0, f_ref)


@pytest.mark.parametrize('bias0', [40.0, 0.8])
def test_coop_early_exit_matches_oracle(eng, bias0):
    """rows emitting the end token at once, or staggered: every workgroup of the group leaves the
    launch at the same step (nets.py:242-243), the rest of the rows read zeros"""
    dims = O.Dims()
    theta = O.make_theta(dims, 8, 4.0, 0.1)
    theta[dims.offsets()['logit.bias'][0]] += np.float32(bias0)
    fc = _fc(130, 55)
    _load(eng, theta, fc)
    eng.set_decode_split(4, 4)
    try:
        assert eng.decode_path(130, 1) == 'coop'
        _, seq, lp = eng.evaluate(2, 0, 1, 0.0, return_seq=True, return_lp=True)
    finally:
        eng.set_decode_split(0, 0)
    seq, lp = seq.cpu().numpy()[0, 0], lp.cpu().numpy()[0, 0]
    oseq, olp, fr = O.decode(dims, theta, fc)
    assert _mismatch(seq, oseq, fr) == []
    if not fr.any():
        assert np.array_equal(seq, oseq)


def test_coop_exact_pass_and_undecided_rows(monkeypatch):
    """the exact tie pass forced on every step (every workgroup of a group runs it), and the bounded
    lse widened so that many rows are undecided: tokens still match the oracle"""
    dims = O.Dims()
    for env, val in (('NICNES_FORCE_EXACT', '1'), ('NICNES_LSE_MARGIN', '1e5')):
        monkeypatch.setenv(env, val)
        e = _engine(max_batch=64, max_members=2, seed=7)
        try:
            theta = O.make_theta(dims, 0, 1.0, 0.0)
            fc = _fc(40, 99)
            _load(e, theta, fc)
            e.set_decode_split(4, 4)
            assert e.decode_path(40, 2) == 'coop'
            _, seq = e.evaluate(3, 0, 2, SIGMA, return_seq=True)
            seq = seq.cpu().numpy()
            assert e.stats()['tie_fallbacks'] > 0 and e.stats()['coop_timeouts'] == 0
            idx = e.noise_indices(3, 0, 2).cpu().numpy()
            for k in range(2):
                for s, sign in enumerate((+1, -1)):
                    oseq, _, fr = O.decode(dims, O.perturb(theta, e._table_np, int(idx[k]), SIGMA, sign), fc)
                    assert _mismatch(seq[k, s], oseq, fr) == [], (env, k, s)
        finally:
            e.close()
        monkeypatch.delenv(env)


@pytest.mark.parametrize('bounded', ['1', '0'], ids=['bounded_lse', 'exact_sum'])
def test_coop_repeated_launches_are_deterministic(monkeypatch, bounded):
    """back-to-back coop launches (counters re-zeroed per launch, uneven progress between groups):
    identical results every time. The lse mode is pinned (NICNES_BOUNDED_LSE): the adaptive policy
    may switch a decode to the exact exp-sum, whose tokens may differ from the bounded one's at
    lse-fragile steps (both equal the reference's up to such a step)."""
    monkeypatch.setenv('NICNES_BOUNDED_LSE', bounded)
    e = _engine(max_batch=128, max_members=64)
    try:
        dims = O.Dims()
        _load(e, O.make_theta(dims, 2, 4.0, 0.1), _fc(128, 8))
        assert e.decode_path(128, 64) == 'coop' or e.n_cu != 256
        ref = [x.clone() for x in e.evaluate(7, 0, 64, SIGMA, return_seq=True)]
        for it in range(5):
            got = e.evaluate(7, 0, 64, SIGMA, return_seq=True)
            bad = (got[1] != ref[1]).nonzero()
            assert bad.shape[0] == 0, (it, bad[:8].tolist(), e.stats())
            assert torch.equal(got[0], ref[0])
        assert e.stats()['coop_timeouts'] == 0
    finally:
        e.close()


def test_coop_needs_a_stage_per_range():
    """the coop path needs a non-empty logit range per workgroup: V1 = 192 (three 64-column stages) takes it at
    S = 2 but not at S = 4, bit-identical to the split path"""
    import nicnes
    e = nicnes.Engine(vocab_size=191, max_batch=128, max_members=4, noise_len=NOISE_LEN, noise_seed=3)
    try:
        e.set_noise_table(O.noise_table(NOISE_LEN, 123))
        rng = np.random.Generator(np.random.PCG64(9))
        theta = (0.05 * rng.standard_normal(e.D)).astype(np.float32)
        _load(e, theta, _fc(128, 77))
        out = {}
        for S, coop in ((4, 1), (2, 1), (2, 0)):
            e.set_decode_split(S, 4)
            e.set_decode_coop(coop)
            out[S, coop] = (e.decode_path(128, 4), e.evaluate(1, 0, 4, SIGMA, return_seq=True, return_lp=True))
        assert out[4, 1][0] == 'split' and out[2, 1][0] == 'coop' and out[2, 0][0] == 'split'
        for a, b in zip(out[2, 1][1], out[2, 0][1]):
            assert torch.equal(a, b)
        assert torch.equal(out[4, 1][1][1], out[2, 0][1][1])     # tokens of the S = 4 split path (empty ranges)
        assert e.stats()['coop_timeouts'] == 0
    finally:
        e.set_decode_coop(1)
        e.set_decode_split(0, 0)
        e.close()
