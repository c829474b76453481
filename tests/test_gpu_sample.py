"""GPU: the sampled fitness modes (Fitness 'sample', 'self_critical', 'sc_loss',
/root/reference/src/captioning/policies.py:22-61,86-193) and their decode, FCModel._sample with
greedy=False (nets.py:210-231: each row draws its token from the softmax with one uniform per row and
logit step), through the C ABI.

Parity: with the draws the reference itself took (tests/golden/decode_sample.npz, replayed numpy
RandomState draws, scripts/make_golden.py) the engine's tokens equal the reference's on every row up to
its first draw within 1e-6 of a cdf boundary (the order p is summed in moves the boundaries by ~1e-7),
and the oracle's (oracle.decode_sample) the same way; fitness against the CIDEr-D / criterion oracle."""
import numpy as np
import pytest

torch = pytest.importorskip('torch')

pytestmark = pytest.mark.gpu

from oracle import oracle as O          # noqa: E402
from oracle import cider_ref as CR      # noqa: E402
from tests.test_oracle_golden import sample_case, U_MARGIN   # noqa: E402

NOISE_LEN = 1 << 23
SIGMA = 0.01


@pytest.fixture(scope='module')
def eng():
    import nicnes
    assert torch.cuda.is_available(), 'GPU tests need a GPU'
    e = nicnes.Engine(max_batch=128, max_members=4, noise_len=NOISE_LEN, noise_seed=7)
    table = O.noise_table(NOISE_LEN, 123)
    e.set_noise_table(table)
    e._table_np = table
    yield e
    e.close()


def _load(eng, theta, fc, seed=11, n_refs=5):
    import nicnes
    import nicnes.synthetic as S
    dims = O.Dims()
    base, _, _ = O.decode(dims, theta, fc)
    gts, df, n = S.build_references(base, dims.vocab_size, seed=seed, n_refs=n_refs, df_sets=256)
    eng.set_theta(theta)
    keys, vals = nicnes.df_table_arrays(df)
    eng.set_df_table(keys, vals, np.log(float(n)))
    eng.set_batch(fc, gts)
    return gts, CR.CiderDOracle(df, n)


_COVERAGE = {}


def _write_coverage():
    import json
    import os
    out = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'gpurun_out')
    os.makedirs(out, exist_ok=True)
    with open(os.path.join(out, 'sample_reference_coverage.json'), 'w') as f:
        json.dump(_COVERAGE, f, indent=1)


def _rows_agree(got, want, stop):
    """tokens equal on each row up to (excluding) its first step where stop[b, t]"""
    n = 0
    for b in range(want.shape[0]):
        for t in range(want.shape[1]):
            if stop[b, t]:
                break
            assert got[b, t] == want[b, t], (b, t, got[b], want[b])
            n += 1
    return n


@pytest.mark.parametrize('name', ['full_xavier', 'full_wc'])
def test_sampled_decode_matches_reference(eng, name):
    """theta itself (sigma = 0, both signs) with the reference's draws: tokens = the reference's and the
    oracle's, sampled log-probs (seq_logprobs) to 5e-6 of the reference's."""
    golden = '%s/golden' % __import__('os').path.dirname(__file__)
    d, theta, fc, g = sample_case(golden, name)
    _load(eng, theta, fc)
    eng.set_fitness_mode('sample')
    try:
        eng.set_sample_draws(np.stack([g['u'], g['u']])[None])
        _, seq, lp = eng.evaluate(1, 0, 1, 0.0, return_seq=True, return_lp=True)
    finally:
        eng.set_sample_draws(None)
        eng.set_fitness_mode('greedy')
    seq, lp = seq.cpu().numpy(), lp.cpu().numpy()
    oseq, olp, ofr = O.decode_sample(d, theta, fc, g['u'])
    for s in range(2):
        stop = (g['u_margin'] < U_MARGIN) | (ofr != 0)
        # compared: each row up to its first draw within U_MARGIN of a cdf boundary (or an oracle-fragile step);
        # the count is fixed by the fixture (full_xavier 532 / 640 = 0.831, full_wc 574 / 640 = 0.897), so a
        # change in what is compared fails here as well as a changed token does
        want_n = int(sum(np.argmax(r) if r.any() else r.size for r in stop))
        n = _rows_agree(seq[0, s], g['seq'], stop)
        assert n == want_n == {'full_xavier': 532, 'full_wc': 574}[name], (n, want_n)
        _COVERAGE[name] = {'positions_compared': n, 'positions': int(seq[0, s].size),
                           'fraction': round(n / seq[0, s].size, 4), 'rows_with_a_fragile_draw': int(stop.any(1).sum()),
                           'u_margin': U_MARGIN}
        _write_coverage()
        _rows_agree(seq[0, s], oseq, ofr != 0)
        live = (~np.cumsum(stop, axis=1).astype(bool)) & (g['logprobs'] != 0)
        assert np.allclose(lp[0, s][live], g['logprobs'][live], rtol=5e-6, atol=5e-6)


def test_sampled_members_match_oracle(eng):
    """perturbed members (theta +- sigma z), seeded draws, one and two slabs: tokens = the oracle's up to the
    first fragile draw; 'sample' fitness = 100 * mean CIDEr-D of the sampled rows (1e-9 relative)."""
    dims = O.Dims()
    theta = O.make_theta(dims, 0, 4.0, 0.1)
    for B in (40, 130):                                     # 130 rows: two 128-row slabs
        fc = np.random.Generator(np.random.PCG64(B)).standard_normal((B, dims.F)).astype(np.float32)
        gts, scorer = _load(eng, theta, fc)
        u = np.random.Generator(np.random.PCG64(5)).random((3, 2, B, dims.T))
        eng.set_fitness_mode('sample')
        try:
            eng.set_sample_draws(u)
            fit, seq = eng.evaluate(4, 0, 3, SIGMA, return_seq=True)
        finally:
            eng.set_sample_draws(None)
            eng.set_fitness_mode('greedy')
        fit, seq = fit.cpu().numpy(), seq.cpu().numpy()
        idx = eng.noise_indices(4, 0, 3).cpu().numpy()
        for k in range(3):
            for s, sign in enumerate((+1, -1)):
                oseq, _, ofr = O.decode_sample(dims, O.perturb(theta, eng._table_np, int(idx[k]), SIGMA, sign), fc,
                                               u[k, s])
                _rows_agree(seq[k, s], oseq, ofr != 0)
                f_ref, _ = CR.rollout_fitness(scorer, seq[k, s], gts)
                assert abs(fit[k, s] - f_ref) <= 1e-9 * max(1.0, abs(f_ref)), (k, s, fit[k, s], f_ref)


def test_self_critical_and_sc_loss(eng):
    """'self_critical' = 100 * mean(sampled row score - greedy row score) = f_sample - f_greedy;
    'sc_loss' = LogFitnessCriterion (fitness.py:12-40) of the sampled log-probs with those per-row
    differences as rewards (the criterion oracle is pinned by tests/golden/fitness_criteria.npz)."""
    dims = O.Dims()
    theta = O.make_theta(dims, 0, 4.0, 0.1)
    B = 40
    fc = np.random.Generator(np.random.PCG64(9)).standard_normal((B, dims.F)).astype(np.float32)
    gts, scorer = _load(eng, theta, fc)
    u = np.random.Generator(np.random.PCG64(6)).random((2, 2, B, dims.T))
    out = {}
    try:
        eng.set_sample_draws(u)
        for mode in ('greedy', 'sample', 'self_critical', 'sc_loss'):
            eng.set_fitness_mode(mode)
            if mode == 'sc_loss':
                out[mode] = tuple(x.cpu().numpy() for x in eng.evaluate(3, 0, 2, SIGMA, return_seq=True,
                                                                        return_lp=True))
            else:
                out[mode] = tuple(x.cpu().numpy() for x in eng.evaluate(3, 0, 2, SIGMA, return_seq=True))
    finally:
        eng.set_sample_draws(None)
        eng.set_fitness_mode('greedy')
    fg, sg = out['greedy']
    fs, ss = out['sample']
    fsc, ssc = out['self_critical']
    fl, sl, lpl = out['sc_loss']
    assert np.array_equal(ss, ssc) and np.array_equal(ss, sl)          # the same draws, the same samples
    assert np.allclose(fsc, fs - fg, rtol=0, atol=1e-9), (fsc, fs - fg)
    for k in range(2):
        for s in range(2):
            _, sc_s = CR.rollout_fitness(scorer, ss[k, s], gts)
            _, sc_g = CR.rollout_fitness(scorer, sg[k, s], gts)
            want = CR.criterion_fitness('sc_loss', lpl[k, s], sl[k, s], np.asarray(sc_s) - np.asarray(sc_g))
            assert abs(fl[k, s] - want) <= 1e-6 * max(1.0, abs(want)), (k, s, fl[k, s], want)
    assert fs.max() > 0.0


def test_engine_draws_are_deterministic_per_iteration(eng):
    """the engine's own draws (no hook): a counter-based hash of (seed, iteration, member, sign, row, step):
    the same iteration repeats exactly, another iteration samples other captions."""
    dims = O.Dims()
    theta = O.make_theta(dims, 0, 1.0, 0.0)
    fc = np.random.Generator(np.random.PCG64(3)).standard_normal((24, dims.F)).astype(np.float32)
    _load(eng, theta, fc)
    eng.set_fitness_mode('sample')
    try:
        a = eng.evaluate(5, 0, 2, SIGMA, return_seq=True)[1].cpu().numpy()
        b = eng.evaluate(5, 0, 2, SIGMA, return_seq=True)[1].cpu().numpy()
        c = eng.evaluate(6, 0, 2, SIGMA, return_seq=True)[1].cpu().numpy()
        d = eng.evaluate(5, 1, 1, SIGMA, return_seq=True)[1].cpu().numpy()
    finally:
        eng.set_fitness_mode('greedy')
    assert np.array_equal(a, b) and not np.array_equal(a, c)
    assert np.array_equal(a[1], d[0])                                  # member 1 draws the same alone
    assert len(np.unique(a[:, :, :, 0])) > 10                          # flat xavier logits: many first words


def test_policy_decodes_every_copy_for_sampled_modes(eng):
    """EnginePolicy.rollout with 'sample': the 5 copies of each image (dataloader.py:175) are decoded, each
    drawing its own tokens (rows_per_image 5 over the 8 unique images held); greedy modes decode one row per
    image."""
    import nicnes.nes as N
    dims = O.Dims()
    theta = O.make_theta(dims, 0, 1.0, 0.0)
    fc = np.random.Generator(np.random.PCG64(3)).standard_normal((8, dims.F)).astype(np.float32)
    gts, _ = _load(eng, theta, fc)
    data = {'fc_feats': np.repeat(fc, 5, 0), 'gts': gts}
    pol = N.EnginePolicy(eng)
    eng.set_fitness_mode('sample')
    try:
        f = pol.rollout(None, data, None)
        assert eng.B == 8 and eng.rpi == 5 and eng.rollout_rows() == 40 and np.isfinite(f)
        _, seq = eng.evaluate(2, 0, 1, SIGMA, return_seq=True)
        seq = seq.cpu().numpy()
        assert seq.shape == (1, 2, 40, dims.T)
        assert any(not np.array_equal(seq[0, 0, 5 * i], seq[0, 0, 5 * i + 1]) for i in range(8))
    finally:
        eng.set_fitness_mode('greedy')
        eng.set_rows_per_image(1)
    assert eng.rollout_rows() == 8


def test_rows_per_image_equals_duplicated_rows(eng):
    """rows_per_image 5 over B unique images = the same batch passed as its 5 B duplicated rows (rows_per_image
    1), with the same draws: tokens, log-probs and fitness identical, for every sampled mode (the self-critical
    baseline then decodes B rows instead of 5 B)."""
    dims = O.Dims()
    theta = O.make_theta(dims, 0, 4.0, 0.1)
    B = 30                                                  # 150 rows: past max_batch (128) and two slabs
    fc = np.random.Generator(np.random.PCG64(21)).standard_normal((B, dims.F)).astype(np.float32)
    gts, _ = _load(eng, theta, fc)
    u = np.random.Generator(np.random.PCG64(22)).random((2, 2, 5 * B, dims.T))
    res = {}
    try:
        eng.set_sample_draws(u)
        for mode in ('sample', 'self_critical', 'sc_loss'):
            eng.set_fitness_mode(mode)
            eng.set_batch(fc, gts)
            eng.set_rows_per_image(5)
            a = [x.cpu().numpy() for x in eng.evaluate(7, 0, 2, SIGMA, return_seq=True, return_lp=True)]
            eng.set_rows_per_image(1)
            eng.set_batch(np.repeat(fc, 5, 0), [g for g in gts for _ in range(5)])
            b = [x.cpu().numpy() for x in eng.evaluate(7, 0, 2, SIGMA, return_seq=True, return_lp=True)]
            res[mode] = (a, b)
    finally:
        eng.set_sample_draws(None)
        eng.set_rows_per_image(1)
        eng.set_fitness_mode('greedy')
    for mode, (a, b) in res.items():
        assert np.array_equal(a[1], b[1]) and np.array_equal(a[2], b[2]), mode
        assert np.allclose(a[0], b[0], rtol=1e-12, atol=1e-12), (mode, a[0], b[0])


def test_sampled_with_member_batches_and_mutation(eng):
    """the sampled decode follows the member -> batch map (single_batch: false) and reads a mutation's
    delta' rows (SM-PROPORTIONAL) like the greedy decode: tokens against the oracle up to the first
    fragile draw, 'sample' fitness against the CIDEr-D oracle on each member's batch."""
    import nicnes
    import nicnes.synthetic as S
    dims = O.Dims()
    theta = O.make_theta(dims, 1, 4.0, 0.1)
    B = 24
    batches = []
    for j in range(2):
        fc = np.random.Generator(np.random.PCG64(40 + j)).standard_normal((B, dims.F)).astype(np.float32)
        base, _, _ = O.decode(dims, theta, fc)
        gts, df, n = S.build_references(base, dims.vocab_size, seed=50 + j, df_sets=256)
        batches.append((fc, gts))
    eng.set_theta(theta)
    keys, vals = nicnes.df_table_arrays(df)
    eng.set_df_table(keys, vals, np.log(float(n)))
    eng.set_batches(batches)
    scorer = CR.CiderDOracle(df, n)
    vec = np.abs(theta).astype(np.float32)
    vec[vec == 0] = np.abs(theta).mean()
    u = np.random.Generator(np.random.PCG64(8)).random((2, 2, B, dims.T))
    mb = [1, 0]
    eng.set_fitness_mode('sample')
    try:
        eng.set_mutation('scale', vec)                       # SM-PROPORTIONAL: delta * |theta'|
        eng.set_sample_draws(u)
        fit, seq = eng.evaluate(3, 0, 2, SIGMA, return_seq=True, member_batch=mb)
    finally:
        eng.set_sample_draws(None)
        eng.set_mutation('plain')
        eng.set_fitness_mode('greedy')
    fit, seq = fit.cpu().numpy(), seq.cpu().numpy()
    idx = eng.noise_indices(3, 0, 2).cpu().numpy()
    for k in range(2):
        fc, gts = batches[mb[k]]
        for s, sign in enumerate((+1, -1)):
            th = O.perturb(theta, eng._table_np, int(idx[k]), SIGMA, sign, ('scale', vec))
            oseq, _, ofr = O.decode_sample(dims, th, fc, u[k, s])
            _rows_agree(seq[k, s], oseq, ofr != 0)
            f_ref, _ = CR.rollout_fitness(scorer, seq[k, s], gts)
            assert abs(fit[k, s] - f_ref) <= 1e-9 * max(1.0, abs(f_ref)), (k, s)


@pytest.mark.parametrize('gain', [1.0, 4.0])
def test_stage_scan_pick_equals_the_full_walk(eng, monkeypatch, gain):
    """The pick from the stage sums (scan the logit loop's per-stage sums to the stage that crosses u * sum(p),
    then walk its 64 logits) against the walk through every stage's logits (NICNES_FORCE_EXACT=1), the same
    terms: tokens and log-probs bit for bit, flat (gain 1) and peaked (gain 4) logits; no row falls back to a
    stage's last id (the sums stopping short of the threshold by rounding)."""
    import nicnes
    dims = O.Dims()
    theta = O.make_theta(dims, 2, gain, 0.1)
    B = 130
    fc = np.random.Generator(np.random.PCG64(77)).standard_normal((B, dims.F)).astype(np.float32)
    u = np.random.Generator(np.random.PCG64(78)).random((3, 2, B, dims.T))
    monkeypatch.setenv('NICNES_FORCE_EXACT', '1')
    ex = nicnes.Engine(max_batch=B, max_members=3, noise_len=NOISE_LEN, noise_seed=7)
    monkeypatch.delenv('NICNES_FORCE_EXACT')
    out = []
    try:
        ex.set_noise_table(eng._table_np)
        for e in (eng, ex):
            _load(e, theta, fc)
            e.set_fitness_mode('sample')
            e.set_sample_draws(u)
            before = e.stats()['sample_stage_fallbacks']
            _, seq, lp = e.evaluate(9, 0, 3, SIGMA, return_seq=True, return_lp=True)
            out.append((seq.cpu().numpy(), lp.cpu().numpy(), e.stats()['sample_stage_fallbacks'] - before))
            e.set_sample_draws(None)
            e.set_fitness_mode('greedy')
    finally:
        ex.close()
    (s1, l1, r1), (s2, l2, r2) = out
    assert eng.stats()['sample_slot_timeouts'] == 0        # every workgroup found a logit slot
    assert np.array_equal(s1, s2)
    assert np.array_equal(l1.view(np.int32), l2.view(np.int32))
    assert r1 == 0 and r2 == 0, (r1, r2)


@pytest.mark.parametrize('gain', [1.0, 4.0])
def test_stage_scan_pick_equals_the_full_walk_at_scale(gain):
    """The same pick-vs-walk identity on a workload where a 4e-5 mis-pick rate cannot hide:
    P = 64 members x 2 signs x 640 rows (128 images x 5 sampled copies) x 16 steps = 1.31 M draws from the
    engine's own counter-based stream, in one launch per engine. Round 4's store-data hazard (the block sums
    zeroed under their own 16-byte store) put ~450 of 10.5 M picks one stage late: ~55 expected here."""
    import nicnes
    dims = O.Dims()
    theta = O.make_theta(dims, 5, gain, 0.1 if gain > 1 else 0.0)
    B, P = 128, 64
    fc = np.random.Generator(np.random.PCG64(81)).standard_normal((B, dims.F)).astype(np.float32)
    table = O.noise_table(NOISE_LEN, 123)
    gts = [np.asarray([[(7 * b + k) % 60 + 1 for k in range(8)] + [0] * 8], np.int32) for b in range(B)]
    keys, vals = nicnes.df_table_arrays({})
    out = []
    for exact in ('0', '1'):
        import os
        os.environ['NICNES_FORCE_EXACT'] = exact
        try:
            e = nicnes.Engine(max_batch=B, max_members=P, noise_len=NOISE_LEN, noise_seed=7)
        finally:
            os.environ.pop('NICNES_FORCE_EXACT', None)
        try:
            e.set_noise_table(table)
            e.set_theta(theta)
            e.set_df_table(keys, vals, np.log(4096.0))
            e.set_batch(fc, gts)
            e.set_fitness_mode('sample')
            e.set_rows_per_image(5)
            _, seq, lp = e.evaluate(3, 0, P, SIGMA, return_seq=True, return_lp=True)
            st = e.stats()
            out.append((seq.cpu().numpy(), lp.cpu().numpy(), st['sample_stage_fallbacks'], st['sample_slot_timeouts']))
        finally:
            e.close()
    (s1, l1, r1, t1), (s2, l2, r2, t2) = out
    assert s1.shape == (P, 2, 5 * B, dims.T)
    assert t1 == t2 == 0 and r1 == 0 and r2 == 0, (r1, r2, t1, t2)
    bad = int((s1 != s2).any(axis=-1).sum())
    assert bad == 0, '%d of %d rows picked differently from the full walk' % (bad, P * 2 * 5 * B)
    assert np.array_equal(l1.view(np.int32), l2.view(np.int32))


def test_logit_slots_are_reused_across_workgroups():
    """More sampled workgroups than logit slots (300 members x 1 slab against n_CU + 16 slots): workgroups that
    start after others finished reuse their slots. Every member's tokens and log-probs equal the same member
    decoded alone (a 3-member launch, no reuse), and no workgroup waited out of a slot."""
    import nicnes
    dims = O.Dims()
    theta = O.make_theta(dims, 4, 4.0, 0.1)
    B, P = 24, 300
    e = nicnes.Engine(max_batch=B, max_members=P, noise_len=NOISE_LEN, noise_seed=7)
    try:
        e.set_noise_table(O.noise_table(NOISE_LEN, 123))
        fc = np.random.Generator(np.random.PCG64(31)).standard_normal((B, dims.F)).astype(np.float32)
        _load(e, theta, fc)
        e.set_fitness_mode('sample')
        _, seq, lp = e.evaluate(11, 0, P, SIGMA, return_seq=True, return_lp=True)
        seq, lp = seq.cpu().numpy(), lp.cpu().numpy()
        for m0 in (0, 148, 297):
            _, s3, l3 = e.evaluate(11, m0, 3, SIGMA, return_seq=True, return_lp=True)
            assert np.array_equal(s3.cpu().numpy(), seq[m0:m0 + 3]), m0
            assert np.array_equal(l3.cpu().numpy().view(np.int32), lp[m0:m0 + 3].view(np.int32)), m0
        assert e.stats()['sample_slot_timeouts'] == 0
    finally:
        e.set_fitness_mode('greedy')
        e.close()
