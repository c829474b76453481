"""GPU properties of the hot path at full fc_caption size (V=9487, E=R=128, F=2048), checked without
re-running the whole decode on the CPU: antithetic symmetry at sigma=0, determinism, member-range
(shard) invariance, noise-index rule bounds, gradient sign/scale linearity, two-slab batches,
'bu' features, and forced exact / near ties in the greedy argmax against the C oracle."""
import numpy as np
import pytest

torch = pytest.importorskip('torch')

pytestmark = pytest.mark.gpu

from oracle import oracle as O          # noqa: E402

NOISE_LEN = 1 << 23
SIGMA = 0.01


@pytest.fixture(scope='module')
def eng():
    import nicnes
    assert torch.cuda.is_available(), 'GPU tests need a GPU'
    e = nicnes.Engine(max_batch=256, max_members=16, noise_len=NOISE_LEN, noise_seed=11)
    table = O.noise_table(NOISE_LEN, 123)
    e.set_noise_table(table)
    e._table_np = table
    yield e
    e.close()


def _load(eng, theta, fc, gts=None):
    import nicnes
    eng.set_theta(theta)
    if gts is None:
        gts = [np.asarray([[(7 * b + k) % 60 + 1 for k in range(8)] + [0] * 8], np.int32) for b in range(fc.shape[0])]
    keys, vals = nicnes.df_table_arrays({})
    eng.set_df_table(keys, vals, np.log(4096.0))
    eng.set_batch(fc, gts)


def _fc(B, seed=1234, bu=False):
    x = np.random.Generator(np.random.PCG64(seed)).standard_normal((B, 2048)).astype(np.float32)
    return np.maximum(x, 0.0) if bu else x


def test_sigma_zero_is_antithetic_symmetric(eng):
    dims = O.Dims()
    _load(eng, O.make_theta(dims, 0, 4.0, 0.1), _fc(64))
    fit, seq = eng.evaluate(3, 0, 6, 0.0, return_seq=True)
    fit, seq = fit.cpu().numpy(), seq.cpu().numpy()
    assert np.array_equal(fit[:, 0], fit[:, 1])
    assert all(np.array_equal(seq[k, s], seq[0, 0]) for k in range(6) for s in range(2))


def test_deterministic_and_shard_invariant(eng):
    dims = O.Dims()
    _load(eng, O.make_theta(dims, 1, 4.0, 0.1), _fc(96))
    f_all, s_all = eng.evaluate(9, 0, 8, SIGMA, return_seq=True)
    f_again, s_again = eng.evaluate(9, 0, 8, SIGMA, return_seq=True)
    f_tail, s_tail = eng.evaluate(9, 5, 3, SIGMA, return_seq=True)
    assert torch.equal(f_all, f_again) and torch.equal(s_all, s_again)
    assert torch.equal(f_all[5:], f_tail) and torch.equal(s_all[5:], s_tail)


def test_noise_index_rule_bounds(eng):
    idx = eng.noise_indices(123456789, 0, 4096).cpu().numpy().astype(np.int64)
    assert np.all(idx % 64 == 0) and idx.min() >= 0 and idx.max() + eng.D <= NOISE_LEN
    ref = [O.noise_index(11, 123456789, m, NOISE_LEN, eng.D) for m in (0, 1, 2047, 4095)]
    assert list(idx[[0, 1, 2047, 4095]]) == ref
    assert len(np.unique(idx)) > 4000            # the rule spreads members over the table


def test_noise_sum_sign_and_scale_linearity(eng):
    P, it = 12, 4
    w = torch.from_numpy(np.random.default_rng(3).standard_normal(P).astype(np.float32)).cuda()
    g = eng.grad_partial(it, 0, P, w, SIGMA)
    g_neg = eng.grad_partial(it, 0, P, -w, SIGMA)
    g_two = eng.grad_partial(it, 0, P, 2 * w, SIGMA)
    assert torch.equal(g_neg, -g) and torch.equal(g_two, 2 * g)
    g_a = eng.grad_partial(it, 0, 7, w[:7], SIGMA).double()
    g_b = eng.grad_partial(it, 7, 5, w[7:], SIGMA).double()
    # shard split: each partial is rounded to fp32 once, so allow a few fp32 ulps of the largest entry
    tol = 4 * float(np.finfo(np.float32).eps) * float(g.abs().max())
    assert float((g_a + g_b - g.double()).abs().max()) <= tol


def test_noise_sum_in_ranges_equals_whole(eng):
    """nicnes_grad_partial_range over 64-aligned cuts of [0, D) rebuilds grad_partial bit for bit (the
    ranges population.py all-reduces while the next one is summed)."""
    P, it = 12, 9
    w = torch.from_numpy(np.random.default_rng(4).standard_normal(P).astype(np.float32)).cuda()
    g = eng.grad_partial(it, 0, P, w, SIGMA)
    cuts = [0, 64 * 3, 64 * 1000, (eng.D // 2) // 64 * 64, eng.D]
    out = torch.full_like(g, float('nan'))
    for j0, j1 in zip(cuts[:-1], cuts[1:]):
        eng.grad_partial_range(it, 0, P, w, SIGMA, j0, j1, out)
    assert torch.equal(out, g)


@pytest.mark.parametrize('B,bu,shape', [(130, False, (0, 0)), (40, True, (0, 0)), (128, True, (0, 0)),
                                         (128, True, (1, 4)), (128, True, (4, 4))],
                         ids=['two_slabs', 'bu_features', 'bu_b128_split', 'bu_b128_fused', 'bu_b128_S4'])
def test_tokens_match_oracle(eng, B, bu, shape):
    """Tokens of one member against the oracle; the 'bu' features (configs[4]) at B = 40 and at the bench's
    B = 128 on the split path, the fused kernel's shape (S = 1) and the coop kernel's (S = 4, G = 4)."""
    dims = O.Dims()
    theta = O.make_theta(dims, 2, 4.0, 0.1)
    fc = _fc(B, 77, bu)
    _load(eng, theta, fc)
    eng.set_decode_split(*shape)
    try:
        _, seq = eng.evaluate(6, 1, 1, SIGMA, return_seq=True)
    finally:
        eng.set_decode_split(0, 0)
    seq = seq.cpu().numpy()[0]
    idx = int(eng.noise_indices(6, 1, 1).cpu().numpy()[0])
    rows = sorted({0, 31, 32, min(127, B - 1), B - 1} | ({128, 129} if B > 128 else set()))
    for s, sign in enumerate((+1, -1)):
        oseq, _, fr = O.decode(dims, O.perturb(theta, eng._table_np, idx, SIGMA, sign), fc[rows])
        for j, b in enumerate(rows):
            for t in range(16):
                if fr[j, t]:
                    break
                assert seq[s, b, t] == oseq[j, t], (sign, b, t)


def _tie_theta(dims, base_theta, fc, copies):
    """Copy the logit row of row 0's first greedy token `tok` to other vocab rows, each with its bias
    raised by k * 2^-22 (about a quarter of the log_softmax tie window at |lse| ~ 10): exact
    (k = 0) and near ties at the maximum, before or after `tok`."""
    seq, _, _ = O.decode(dims, base_theta, fc[:1])
    tok = int(seq[0, 0])
    th = base_theta.copy()
    o = dims.offsets()
    V1, R = dims.vocab_size + 1, dims.R
    lw = th[o['logit.weight'][0]:o['logit.weight'][0] + V1 * R].reshape(V1, R)
    lb = th[o['logit.bias'][0]:o['logit.bias'][0] + V1]
    for where, k in copies:
        dst = {'lower': max(tok // 2, 1), 'higher': min(tok + 8, V1 - 1), 'higher2': min(tok + 16, V1 - 1)}[where]
        lw[dst] = lw[tok]
        lb[dst] = lb[tok] + np.float32(k * 2.0 ** -22)
    return th, tok


@pytest.mark.parametrize('copies', [
    [('lower', 0)], [('lower', 1)], [('higher', 1)], [('higher', 1), ('higher2', 2)],
], ids=['exact_lower', 'near_lower', 'near_higher', 'triple_higher'])
def test_forced_ties_follow_oracle(eng, copies):
    dims = O.Dims()
    base = O.make_theta(dims, 4, 4.0, 0.1)
    fc = _fc(32, 91)
    th, tok = _tie_theta(dims, base, fc, copies)
    _load(eng, th, fc)
    _, seq = eng.evaluate(2, 0, 1, 0.0, return_seq=True)       # sigma 0: both signs decode th
    seq = seq.cpu().numpy()[0, 0]
    oseq, _, fr = O.decode(dims, th, fc)
    for b in range(fc.shape[0]):
        for t in range(16):
            if fr[b, t]:
                break
            assert seq[b, t] == oseq[b, t], (b, t)


@pytest.mark.parametrize('S,G,coop', [(1, 4, 1), (4, 4, 0), (4, 4, 1), (4, 2, 0), (1, 2, 0)],
                         ids=['fused_2slabs', 'split_2slabs', 'coop_2slabs', 'split_G2_3slabs', 'fused_G2_3slabs'])
def test_logprobs_after_a_slab_exit_match_oracle(eng, S, G, coop):
    """seq_logprobs of a batch that spans several slabs (B = 130): the reference writes the greedy
    log-prob of every row, finished or not, until the WHOLE batch has finished (nets.py:240-243) and
    leaves zeros after. With log-prob output the engine runs every slab to T and zeroes the steps after
    the batch's last finishing step; staggered finishing (logit.bias[0] raised) makes slabs finish at
    different steps. Every row and step against the oracle's whole-batch decode (1e-5, up to a row's
    first lse-fragile step), tokens end to end."""
    dims = O.Dims()
    theta = O.make_theta(dims, 8, 4.0, 0.1)
    theta[dims.offsets()['logit.bias'][0]] += np.float32(0.8)
    fc = _fc(130, 55)
    _load(eng, theta, fc)
    eng.set_decode_split(S, G)
    eng.set_decode_coop(coop)
    try:
        _, seq, lp = eng.evaluate(2, 0, 1, 0.0, return_seq=True, return_lp=True)
        _, seq_nolp = eng.evaluate(2, 0, 1, 0.0, return_seq=True)
    finally:
        eng.set_decode_split(0, 0)
        eng.set_decode_coop(1)
    seq, lp = seq.cpu().numpy()[0, 0], lp.cpu().numpy()[0, 0]
    assert np.array_equal(seq, seq_nolp.cpu().numpy()[0, 0])       # the run to T changes no token
    oseq, olp, fr = O.decode(dims, theta, fc)
    fin = np.array([np.argmax(r == 0) if (r == 0).any() else 16 for r in oseq])
    slab = 32 * G
    firsts = [fin[i:i + slab].max() for i in range(0, 130, slab)]
    assert len(set(firsts)) > 1, firsts                             # the slabs do finish at different steps
    assert fin.max() < 15                                           # and the batch before T
    ok = ~np.cumsum(fr, 1).astype(bool)
    assert np.array_equal(seq[ok], oseq[ok])
    assert np.abs(lp[ok] - olp[ok]).max() <= 1e-5
    assert (lp[:, fin.max() + 1:] == 0).all() and (olp[:, fin.max() + 1:] == 0).all()


def test_last_decode_lse_mode_reports_the_instantiation(eng):
    """nicnes_last_decode_lse (bench.py's PMC attribution): a greedy-only decode at xavier theta runs the pair-bounded
    lse, one with log-probs written the exact exp-sum; the tokens agree. (A fresh handle: the module engine's adaptive
    policy may be in an exact stretch after the forced-tie tests.)"""
    import nicnes
    e = nicnes.Engine(max_batch=32, max_members=2, noise_len=NOISE_LEN, noise_seed=11)
    try:
        e.set_noise_table(eng._table_np)
        dims = O.Dims()
        _load(e, O.make_theta(dims, 0, 1.0, 0.0), _fc(32))
        _, s_b = e.evaluate(5, 0, 2, SIGMA, return_seq=True)
        assert e.last_decode_bounded()
        _, s_e, _ = e.evaluate(5, 0, 2, SIGMA, return_seq=True, return_lp=True)
        assert not e.last_decode_bounded()
        assert torch.equal(s_b, s_e)
    finally:
        e.close()
