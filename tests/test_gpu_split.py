"""GPU parity of the split decode path (nicnes_decode_logit_kernel / nicnes_decode_cell_kernel):
one member's step spread over S workgroups (vocabulary ranges for the logits, unit blocks for the
cell) and 64-row slabs (G = 2) for batches of <= 64 images, against the C oracle. Every test runs
twice: with the coop path on (nicnes_decode_coop_kernel takes the G = 4, S = 2 / 4 shapes in one
launch) and off (two launches per step for every split shape).

Covers the shapes the automatic rule picks for BASELINE.json configs[1] (pop=64, B=128 -> S=4) and
mscoco_nes.json's batch_size 64 (G=2), forced shapes from the fused kernel (G=4, S=1) up to S=16,
the early exit (nets.py:242-243) through the split alive chain, the exact tie pass and forced
near-ties. Tokens are bit-exact against the oracle except after a step it marks lse-fragile;
CIDEr-D fitness to 1e-9 relative."""
import numpy as np
import pytest

torch = pytest.importorskip('torch')

pytestmark = pytest.mark.gpu

from oracle import oracle as O          # noqa: E402
from oracle import cider_ref as CR      # noqa: E402

NOISE_LEN = 1 << 23
SIGMA = 0.01
SHAPES = [(4, 1), (4, 2), (4, 4), (4, 16), (2, 1), (2, 4), (2, 8)]


@pytest.fixture(scope='module', params=[1, 0], ids=['coop', 'nocoop'])
def eng(request):
    import nicnes
    assert torch.cuda.is_available(), 'GPU tests need a GPU'
    e = nicnes.Engine(max_batch=128, max_members=64, noise_len=NOISE_LEN, noise_seed=5)
    table = O.noise_table(NOISE_LEN, 123)
    e.set_noise_table(table)
    e._table_np = table
    e.set_decode_coop(request.param)
    yield e
    assert e.stats()['coop_timeouts'] == 0
    e.set_decode_split(0, 0)
    e.close()


def _load(eng, theta, fc, gts=None, df=None, ref_len_raw=4096):
    import nicnes
    eng.set_theta(theta)
    if gts is None:
        gts = [np.asarray([[(7 * b + k) % 60 + 1 for k in range(8)] + [0] * 8], np.int32) for b in range(fc.shape[0])]
    keys, vals = nicnes.df_table_arrays(df or {})
    eng.set_df_table(keys, vals, np.log(float(ref_len_raw)))
    eng.set_batch(fc, gts)


def _fc(B, seed=1234):
    return np.random.Generator(np.random.PCG64(seed)).standard_normal((B, 2048)).astype(np.float32)


def _mismatch(gpu, ora, fragile):
    """rows whose tokens differ before the first lse-fragile step"""
    bad = []
    for b in range(ora.shape[0]):
        for t in range(ora.shape[1]):
            if fragile[b, t]:
                break
            if gpu[b, t] != ora[b, t]:
                bad.append((b, t))
                break
    return bad


_oracle_cache = {}


def _oracle(theta_key, theta, table, idx, fc, sign):
    key = (theta_key, idx, fc.shape[0], sign)
    if key not in _oracle_cache:
        _oracle_cache[key] = O.decode(O.Dims(), O.perturb(theta, table, idx, SIGMA, sign), fc)
    return _oracle_cache[key]


@pytest.mark.parametrize('B', [40, 100])
@pytest.mark.parametrize('G,S', SHAPES, ids=['G%dS%d' % s for s in SHAPES])
def test_shapes_tokens_match_oracle(eng, G, S, B):
    dims = O.Dims()
    theta = O.make_theta(dims, 6, 4.0, 0.1)
    fc = _fc(B, 321)
    _load(eng, theta, fc)
    eng.set_decode_split(S, G)
    try:
        assert eng.decode_shape(B, 2) == (G, (B + 32 * G - 1) // (32 * G), S)
        _, seq, lp = eng.evaluate(4, 3, 2, SIGMA, return_seq=True, return_lp=True)
    finally:
        eng.set_decode_split(0, 0)
    seq, lp = seq.cpu().numpy(), lp.cpu().numpy()
    idx = eng.noise_indices(4, 3, 2).cpu().numpy()
    for k in range(2):
        for s, sign in enumerate((+1, -1)):
            oseq, olp, fr = _oracle('wc6', theta, eng._table_np, int(idx[k]), fc, sign)
            assert _mismatch(seq[k, s], oseq, fr) == [], (G, S, B, k, s)
            m = np.concatenate([np.ones((B, 1), bool), oseq[:, :-1] > 0], 1) & ~np.cumsum(fr, 1).astype(bool)
            assert np.abs(lp[k, s][m] - olp[m]).max() <= 1e-5


def _bench_like(eng, B, seed_fc=1234):
    """xavier theta (the bench's init) plus references derived from its own base caption"""
    import nicnes.synthetic as S
    dims = O.Dims()
    theta = S.init_theta(S.Dims(), 0)
    fc = _fc(B, seed_fc)
    base, _, _ = O.decode(dims, theta, fc)
    gts, df, n = S.build_references(base, dims.vocab_size, seed=4321, n_refs=5, df_sets=512)
    _load(eng, theta, fc, gts, df, n)
    return theta, fc, gts, df, n


@pytest.mark.parametrize('B,want', [(128, (4, 1, 4)), (64, (2, 1, 4))], ids=['configs1_pop64_B128', 'pop64_B64'])
def test_pop64_auto_shape_tokens_and_fitness(eng, B, want):
    """64 members in one launch with the automatic shape (configs[1]; B = 64 is mscoco_nes.json's
    batch_size): 8 members against the oracle decode and scorer, the rest against the fused path."""
    theta, fc, gts, df, n = _bench_like(eng, B)
    P = 64
    shape = eng.decode_shape(B, P)
    if eng.n_cu == 256:
        assert shape == want
        assert eng.decode_path(B, P) == ('coop' if (B == 128 and eng.coop_mode) else 'split')
    fit, seq = eng.evaluate(1, 0, P, SIGMA, return_seq=True)
    fit, seq = fit.cpu().numpy(), seq.cpu().numpy()
    idx = eng.noise_indices(1, 0, P).cpu().numpy()
    scorer = CR.CiderDOracle(df, n)
    for i in np.linspace(0, P - 1, 8).astype(int):
        for s, sign in enumerate((+1, -1)):
            oseq, _, fr = O.decode(O.Dims(), O.perturb(theta, eng._table_np, int(idx[i]), SIGMA, sign), fc)
            assert _mismatch(seq[i, s], oseq, fr) == [], (i, s)
            f_ref, _ = CR.rollout_fitness(scorer, seq[i, s], gts)
            assert abs(fit[i, s] - f_ref) <= 1e-9 * max(1.0, f_ref), (i, s, fit[i, s], f_ref)
    assert np.isfinite(fit).all() and fit.std() > 0
    # the fused kernel on the same members: tokens may differ only where the oracle marks a
    # step lse-fragile (the merge sums exp in another order); at this theta none differ
    eng.set_decode_split(1, 4)
    try:
        fit1, seq1 = eng.evaluate(1, 0, P, SIGMA, return_seq=True)
    finally:
        eng.set_decode_split(0, 0)
    same = (seq1.cpu().numpy() == seq).all(axis=(2, 3)).mean()
    assert same >= 0.95, same


def test_split_shard_invariance(eng):
    dims = O.Dims()
    _load(eng, O.make_theta(dims, 1, 4.0, 0.1), _fc(96))
    eng.set_decode_split(4, 4)
    try:
        f_all, s_all = eng.evaluate(9, 0, 8, SIGMA, return_seq=True)
        f_tail, s_tail = eng.evaluate(9, 5, 3, SIGMA, return_seq=True)
        f_again = eng.evaluate(9, 0, 8, SIGMA)
    finally:
        eng.set_decode_split(0, 0)
    assert torch.equal(f_all, f_again)
    assert torch.equal(f_all[5:], f_tail) and torch.equal(s_all[5:], s_tail)


@pytest.mark.parametrize('bias0', [40.0, 1.0, 0.8])
@pytest.mark.parametrize('G,S', [(4, 4), (2, 4), (4, 1), (2, 1)], ids=['G4S4', 'G2S4', 'fused', 'fused_G2'])
def test_early_exit_matches_oracle(eng, G, S, bias0):
    """logit.bias[0] raised so rows emit the end token at step 1 (all finish at once), or at
    staggered steps: the split alive chain must stop exactly where the reference stops
    (nets.py:242-243) and leave zeros after it."""
    dims = O.Dims()
    theta = O.make_theta(dims, 8, 4.0, 0.1)
    theta[dims.offsets()['logit.bias'][0]] += np.float32(bias0)
    fc = _fc(48, 55)
    _load(eng, theta, fc)
    eng.set_decode_split(S, G)
    try:
        _, seq, lp = eng.evaluate(2, 0, 1, 0.0, return_seq=True, return_lp=True)
    finally:
        eng.set_decode_split(0, 0)
    seq, lp = seq.cpu().numpy()[0, 0], lp.cpu().numpy()[0, 0]
    oseq, olp, fr = O.decode(dims, theta, fc)
    assert _mismatch(seq, oseq, fr) == []
    fin = np.array([np.argmax(r == 0) if (r == 0).any() else 16 for r in oseq])
    assert fin.max() < 16                                  # the batch finishes before T
    if not fr.any():
        assert np.array_equal(seq, oseq)
        assert np.abs(lp - olp).max() <= 1e-5              # zeros past the global exit, as the reference


@pytest.mark.parametrize('coop', [1, 0], ids=['coop', 'nocoop'])
def test_split_exact_tie_pass_matches_oracle(monkeypatch, coop):
    """The exact second pass forced on every step of the split path (every cell workgroup of a
    member runs it): tokens still match the oracle."""
    import nicnes
    monkeypatch.setenv('NICNES_FORCE_EXACT', '1')
    e = nicnes.Engine(max_batch=64, max_members=2, noise_len=NOISE_LEN, noise_seed=7)
    e.set_decode_coop(coop)
    try:
        table = O.noise_table(NOISE_LEN, 123)
        e.set_noise_table(table)
        dims = O.Dims()
        theta = O.make_theta(dims, 5, 4.0, 0.1)
        fc = _fc(40, 4321)
        _load(e, theta, fc)
        idx = int(e.noise_indices(3, 0, 1).cpu().numpy()[0])
        for G, S in ((4, 4), (2, 2)):
            e.set_decode_split(S, G)
            _, seq = e.evaluate(3, 0, 1, SIGMA, return_seq=True)
            seq = seq.cpu().numpy()
            for s, sign in enumerate((+1, -1)):
                oseq, _, fr = O.decode(dims, O.perturb(theta, table, idx, SIGMA, sign), fc)
                assert _mismatch(seq[0, s], oseq, fr) == [], (G, S, s)
        assert e.stats()['tie_fallbacks'] >= 32
    finally:
        e.close()


@pytest.mark.parametrize('G,S', [(4, 4), (2, 4)], ids=['G4S4', 'G2S4'])
def test_split_forced_ties_follow_oracle(eng, G, S):
    """exact and near ties at the maximum placed on either side of a vocabulary range boundary"""
    dims = O.Dims()
    base = O.make_theta(dims, 4, 4.0, 0.1)
    fc = _fc(32, 91)
    seq0, _, _ = O.decode(dims, base, fc[:1])
    tok = int(seq0[0, 0])
    V1, R = dims.vocab_size + 1, dims.R
    o = dims.offsets()
    nst = (V1 + 63) // 64
    # the first stage of another workgroup's vocabulary range, before and after tok
    bounds = [64 * (q * nst // S) for q in range(1, S)]
    dsts = [b for b in bounds if b != tok][:2] + [max(tok // 2, 1)]
    for k_tie in (0, 1):
        th = base.copy()
        lw = th[o['logit.weight'][0]:o['logit.weight'][0] + V1 * R].reshape(V1, R)
        lb = th[o['logit.bias'][0]:o['logit.bias'][0] + V1]
        for d in dsts:
            lw[d] = lw[tok]
            lb[d] = lb[tok] + np.float32(k_tie * 2.0 ** -22)
        _load(eng, th, fc)
        eng.set_decode_split(S, G)
        try:
            _, seq = eng.evaluate(2, 0, 1, 0.0, return_seq=True)
        finally:
            eng.set_decode_split(0, 0)
        oseq, _, fr = O.decode(dims, th, fc)
        assert _mismatch(seq.cpu().numpy()[0, 0], oseq, fr) == [], (k_tie, dsts)


@pytest.mark.parametrize('S,G', [(4, 4), (1, 4), (4, 2), (1, 2)], ids=['split_G4S4', 'fused', 'split_G2S4', 'fused_G2'])
def test_decode_streams_do_not_change_results(eng, S, G):
    """members split over 1..4 streams (nicnes_set_decode_streams; 7 members split unevenly, ragged
    100-row slabs): fitness, tokens and log-probs bit-identical to the one-stream decode"""
    dims = O.Dims()
    _load(eng, O.make_theta(dims, 6, 4.0, 0.1), _fc(100, 77))
    eng.set_decode_split(S, G)
    out = {}
    try:
        for n in (1, 2, 3, 4):
            eng.set_decode_streams(n)
            fit, seq, lp = eng.evaluate(6, 2, 7, SIGMA, return_seq=True, return_lp=True)
            out[n] = (fit.clone(), seq.clone(), lp.clone())
    finally:
        eng.set_decode_streams(0)
        eng.set_decode_split(0, 0)
    for n in (2, 3, 4):
        for a, b in zip(out[1], out[n]):
            assert torch.equal(a, b), n
