"""Safe / proportional mutations on the GPU (PolicyNet.evolve, src/algorithm/nets.py:83-119): with
nicnes_set_mutation the members evaluate theta +/- delta', delta' = fp32(sigma * z) / s (SM-G-SUM,
SM-VECTOR) or fp32(sigma * z) * |theta'| (SM-PROPORTIONAL), and the weighted noise sum and
nicnes_noise_vectors use the same delta'. Checked against the oracle (oracle.member_delta):
tokens and CIDEr-D fitness of every member on the fused and the split decode, delta' bit for bit,
the noise sum bit for bit (fp64 accumulation in member order, one rounding)."""
import numpy as np
import pytest

torch = pytest.importorskip('torch')

pytestmark = pytest.mark.gpu

from oracle import oracle as O          # noqa: E402
from oracle import cider_ref as CR      # noqa: E402

NOISE_LEN = 1 << 23
SIGMA = 0.01
SEED, IT = 6, 9


def _vector(mode, theta, D):
    from nicnes import mutations as MU
    if mode == 'scale':
        return MU.proportional_vector(theta).numpy()
    # a sensitivity-like vector: clamped at the underflow and divided by it (values >= 1)
    s = np.random.Generator(np.random.PCG64(5)).gamma(0.5, 4.0, D).astype(np.float32)
    return MU.clamp_calc(torch.from_numpy(s), 0.1).numpy()


@pytest.mark.parametrize('shape', [(1, 4), (4, 2)], ids=['fused', 'split_G2S4'])
@pytest.mark.parametrize('mode', ['divide', 'scale'])
def test_mutated_members_match_oracle(mode, shape):
    import nicnes
    import nicnes.synthetic as S
    dims = O.Dims()
    theta = O.make_theta(dims, 4, 4.0, 0.1)
    theta[:dims.E * dims.F:7] = 0.0                      # exact zeros: SM-PROPORTIONAL's mean replacement
    B, P = 24, 5
    fc = np.random.Generator(np.random.PCG64(31)).standard_normal((B, dims.F)).astype(np.float32)
    base, _, _ = O.decode(dims, theta, fc)
    gts, df, n = S.build_references(base, dims.vocab_size, seed=3, n_refs=5, df_sets=128)
    table = O.noise_table(NOISE_LEN, 123)
    vec = _vector(mode, theta, dims.D)
    mut = (mode, vec)
    e = nicnes.Engine(max_batch=B, max_members=P, noise_len=NOISE_LEN, noise_seed=SEED)
    try:
        e.set_noise_table(table)
        keys, vals = nicnes.df_table_arrays(df)
        e.set_df_table(keys, vals, np.log(float(n)))
        e.set_theta(theta)
        e.set_batch(fc, gts)
        e.set_decode_split(*shape)
        e.set_mutation(mode, vec)
        fit, seq = e.evaluate(IT, 0, P, SIGMA, return_seq=True)
        fit, seq = fit.cpu().numpy(), seq.cpu().numpy()
        dv = e.noise_vectors(IT, 0, P, SIGMA).cpu().numpy()
        scorer = CR.CiderDOracle(df, n)
        idx = [O.noise_index(SEED, IT, k, NOISE_LEN, dims.D) for k in range(P)]
        for k in range(P):
            want = O.member_delta(table, idx[k], SIGMA, dims.D, mut)
            assert np.array_equal(dv[k], want), k
            assert not np.array_equal(want, O.member_delta(table, idx[k], SIGMA, dims.D))
            for s, sign in enumerate((+1, -1)):
                oseq, _, fr = O.decode(dims, O.perturb(theta, table, idx[k], SIGMA, sign, mut), fc)
                ok = fr.any(axis=1) | (seq[k, s] == oseq).all(axis=1)
                assert ok.all(), (k, s)
                if not fr.any():
                    f_ref = CR.rollout_fitness(scorer, oseq, gts)[0]
                    assert abs(fit[k, s] - f_ref) <= 1e-9 * max(1.0, f_ref), (k, s, fit[k, s], f_ref)
        w = torch.linspace(-0.5, 0.5, P, dtype=torch.float32, device=e.device)
        g = e.grad_partial(IT, 0, P, w, SIGMA).cpu().numpy()
        acc = np.zeros(dims.D, np.float64)
        for k in range(P):
            acc += np.float64(w[k].item()) * O.member_delta(table, idx[k], SIGMA, dims.D, mut).astype(np.float64)
        assert np.array_equal(g, acc.astype(np.float32))
        # plain again: the table's delta
        e.set_mutation('plain')
        dv0 = e.noise_vectors(IT, 0, 1, SIGMA).cpu().numpy()
        assert np.array_equal(dv0[0], np.float32(SIGMA) * table[idx[0]: idx[0] + dims.D])
    finally:
        e.close()


SENS_RTOL = 5e-5     # GPU sensitivity vs the torch-autograd oracle: fp32 sums in another order (measured <= 1.0e-5)


def _sens_close(gpu, ref):
    """elementwise |gpu - ref| <= SENS_RTOL * |ref| + 1e-6 * max|ref| (the vector spans many decades; near-zero
    entries carry only absolute error)"""
    gpu, ref = np.asarray(gpu, np.float64), np.asarray(ref, np.float64)
    err = np.abs(gpu - ref)
    bound = SENS_RTOL * np.abs(ref) + 1e-6 * np.abs(ref).max()
    return bool((err <= bound).all()), float((err / np.maximum(np.abs(ref), 1e-30))[np.abs(ref) > 1e-3 * np.abs(ref).max()].max())


@pytest.mark.parametrize('theta_kind,rows', [('xavier', 8), ('wc', 16), ('wc', 41)])
def test_gpu_sensitivity_matches_oracle(theta_kind, rows):
    """nicnes_sum_sensitivity (95 backward passes batched on the GPU, the square sums fused into the MFMA tile
    kernels) against the torch-autograd restatement oracle/sensitivity_ref.py, itself bit-exact with the
    reference's Sensitivity.calc_sensitivity (tests/golden/mutations.npz): the raw vector and the clamped one
    (underflow 0.1, mscoco_nes.json). Bit-identical from call to call (no atomics: ADVICE r03)."""
    import nicnes
    from nicnes import mutations as MU
    from oracle import sensitivity_ref as SR
    dims = O.Dims()
    theta = O.make_theta(dims, 0, 1.0, 0.0) if theta_kind == 'xavier' else O.make_theta(dims, 3, 4.0, 0.1)
    fc = np.random.Generator(np.random.PCG64(77)).standard_normal((rows + 4, dims.F)).astype(np.float32)
    e = nicnes.Engine(max_batch=rows + 4, max_members=2, noise_len=NOISE_LEN, noise_seed=0)
    try:
        e.set_noise_table(O.noise_table(NOISE_LEN, 123))
        e.set_theta(theta)
        e.set_df_table(np.zeros(0, np.uint64), np.zeros(0), np.log(64.0))
        e.set_batch(fc, [np.zeros((1, dims.T), np.int32)] * fc.shape[0])
        raw = e.sum_sensitivity(rows).cpu().numpy()
        clamped = e.sum_sensitivity(rows, 0.1).cpu().numpy()
        assert np.array_equal(e.sum_sensitivity(rows).cpu().numpy(), raw)
    finally:
        e.close()
    ref = SR.sum_sensitivity((dims.vocab_size + 1, dims.E, dims.R, dims.F), theta, fc[:rows], rows).numpy()
    ok, worst = _sens_close(raw, ref)
    assert ok, worst
    ok, worst = _sens_close(clamped, MU.clamp_calc(torch.from_numpy(ref), 0.1).numpy())
    assert ok, worst
    print('max relative error over entries >= 1e-3 max: %.3g' % worst)


@pytest.mark.parametrize('vocab,theta_kind', [(999, 'wc'), (511, 'wc'), (511, 'xavier'), (127, 'xavier')])
def test_gpu_sensitivity_small_vocabulary(vocab, theta_kind):
    """a vocabulary below ~8,400 words has fewer seeds than the embedding kernels' 8 k lanes x 12 cover
    (K = V1 / 100 + 1 = 11 at 999 words, 6 at 511, 2 at 127): the lanes past K must not read beyond dX. The vector
    matches the restatement oracle within the full-vocabulary bar. (Below ~500 words with the peaked theta, and at
    63 words with either, single-seed square sums amplify fp32 summation-order rounding to 1-2x the bar in a few
    i2h entries: scripts/debug_sens_vocab.py; the reference vocabulary is 9,487 words.)"""
    import nicnes
    from oracle import sensitivity_ref as SR
    dims = O.Dims(vocab_size=vocab)
    theta = O.make_theta(dims, 3, 4.0, 0.1) if theta_kind == 'wc' else O.make_theta(dims, 0, 1.0, 0.0)
    rows = 12
    fc = np.random.Generator(np.random.PCG64(78)).standard_normal((rows, dims.F)).astype(np.float32)
    e = nicnes.Engine(vocab_size=vocab, max_batch=rows, max_members=2, noise_len=NOISE_LEN, noise_seed=0)
    try:
        e.set_noise_table(O.noise_table(NOISE_LEN, 123))
        e.set_theta(theta)
        e.set_df_table(np.zeros(0, np.uint64), np.zeros(0), np.log(64.0))
        e.set_batch(fc, [np.zeros((1, dims.T), np.int32)] * rows)
        raw = e.sum_sensitivity(rows).cpu().numpy()
        assert np.array_equal(e.sum_sensitivity(rows).cpu().numpy(), raw)
    finally:
        e.close()
    ref = SR.sum_sensitivity((dims.vocab_size + 1, dims.E, dims.R, dims.F), theta, fc, rows).numpy()
    ok, worst = _sens_close(raw, ref)
    assert ok, worst


@pytest.mark.parametrize('twin', ['before', 'after'])
def test_sensitivity_greedy_tokens_at_planted_ties(twin):
    """the SM-G-SUM forward picks its own greedy tokens (sens_greedy). For every distinct first token a
    of the batch a twin row b = a - 1 or a + 1 is planted: logit row b = row a, bias b one ulp above bias a, so b
    ties a (equal logits, or one ulp of z apart: well inside the ulp(lse) / 2 window of log_softmax) wherever a
    wins. torch.max over the log-probs then takes the first index, min(a, b) (the oracle decode confirms it on
    every row); an argmax over the raw logits would take b when it is one ulp higher. The GPU vector must equal
    the reference-order restatement there too (a different token changes a row's whole contribution)."""
    import nicnes
    from oracle import sensitivity_ref as SR
    dims = O.Dims()
    rows = 16
    theta = O.make_theta(dims, 5, 2.0, 0.05)
    fc = np.random.Generator(np.random.PCG64(79)).standard_normal((rows, dims.F)).astype(np.float32)
    seq, _, _ = O.decode(dims, theta, fc)
    ow, _ = dims.offsets()['logit.weight']
    ob, _ = dims.offsets()['logit.bias']
    R = dims.R
    th = theta.copy()
    winners = sorted(set(int(a) for a in seq[:, 0]))
    used, twin_of = set(winners), {}
    for a in winners:
        b = a - 1 if twin == 'before' else a + 1
        if b < 1 or b >= dims.V1 or b in used:
            continue
        used.add(b)
        twin_of[a] = b
        th[ow + b * R: ow + (b + 1) * R] = th[ow + a * R: ow + (a + 1) * R]
        th[ob + b] = np.nextafter(th[ob + a], np.float32(np.inf))
    seq2, _, _ = O.decode(dims, th, fc)
    assert len(twin_of) >= 8
    assert np.array_equal(seq2[:, 0], [min(a, twin_of.get(a, a)) for a in seq[:, 0]])   # first-index rule
    e = nicnes.Engine(max_batch=rows, max_members=2, noise_len=NOISE_LEN, noise_seed=0)
    try:
        e.set_noise_table(O.noise_table(NOISE_LEN, 123))
        e.set_theta(th)
        e.set_df_table(np.zeros(0, np.uint64), np.zeros(0), np.log(64.0))
        e.set_batch(fc, [np.zeros((1, dims.T), np.int32)] * rows)
        raw = e.sum_sensitivity(rows).cpu().numpy()
    finally:
        e.close()
    ref = SR.sum_sensitivity((dims.vocab_size + 1, dims.E, dims.R, dims.F), th, fc, rows).numpy()
    ok, worst = _sens_close(raw, ref)
    assert ok, worst


def test_safe_mutation_master_trajectory_matches_oracle_engine():
    """EngineMaster.run with model_options.safe_mutations 'SM-G-SUM': the engine's GPU sensitivity drives the
    GPU transform; two iterations match the oracle engine run by the same master. The per-iteration vector
    is checked against the oracle's (SENS_RTOL), then the oracle engine is handed the GPU's vector, so that
    everything after it (transform, decode, fitness, ranks, noise sum, Adam) is compared exactly."""
    import nicnes
    import nicnes.synthetic as S
    from nicnes import config as C, master as M
    from tests.cpu_engine import OracleEngine
    dims = O.Dims()
    theta = O.make_theta(dims, 0, 4.0, 0.1)
    fc = np.random.Generator(np.random.PCG64(1234)).standard_normal((8, dims.F)).astype(np.float32)
    base, _, _ = O.decode(dims, theta, fc)
    gts, df, n = S.build_references(base, dims.vocab_size, seed=9, n_refs=5, df_sets=128)
    table = O.noise_table(NOISE_LEN, 123)
    P = 4
    spec = C.ExperimentSpec({'algorithm': 'nic_nes', 'nb_offspring': P,
                             'config': {'noise_stdev': 0.01, 'batch_size': 8, 'l2coeff': 1e-3, 'snapshot_freq': 0,
                                        'single_batch': True},
                             'policy_options': {'net': 'fc_caption', 'fitness': 'greedy',
                                                'model_options': {'safe_mutations': 'SM-G-SUM',
                                                                  'safe_mutation_underflow': 0.1}},
                             'optimizer_options': {'type': 'adam', 'args': {'stepsize': 1e-3}}})
    e = nicnes.Engine(max_batch=8, max_members=P, noise_len=NOISE_LEN, noise_seed=0)
    try:
        e.set_noise_table(table)
        keys, vals = nicnes.df_table_arrays(df)
        e.set_df_table(keys, vals, np.log(float(n)))
        batch = {'fc_feats': np.repeat(fc, 5, axis=0), 'gts': gts}
        gpu_vectors = []
        gpu_sens = e.sum_sensitivity
        e.sum_sensitivity = lambda rows, uf: gpu_vectors.append(gpu_sens(rows, uf).clone()) or gpu_vectors[-1]
        gpu = M.EngineMaster(spec, e, theta=theta)
        gpu.run([batch], max_iterations=2)
        ora_e = OracleEngine(dims, theta, fc, gts, df, n, table, noise_seed=0)
        ora_sens = ora_e.sum_sensitivity
        replay = list(gpu_vectors)

        def handed(rows, uf):
            ok, worst = _sens_close(replay[0].cpu().numpy(), ora_sens(rows, uf).numpy())
            assert ok, worst
            return replay.pop(0).cpu()
        ora_e.sum_sensitivity = handed
        ora = M.EngineMaster(spec, ora_e, theta=theta)
        ora.run([batch], max_iterations=2)
        assert len(gpu_vectors) == 2 and not replay and e.mutation_mode == 1
        for a, b in zip(gpu.stats, ora.stats):
            assert abs(a['score_mean'] - b['score_mean']) <= 1e-9 * max(1.0, abs(b['score_mean']))
        assert np.allclose(e.theta()[0].cpu().numpy(), ora_e.adam.theta, rtol=1e-6, atol=1e-12)
    finally:
        e.close()


def test_proportional_vector_formed_on_the_device_equals_the_host_one():
    """nicnes_set_mutation_proportional: |theta'| formed from the handle's own theta on the GPU (exact zeros of
    either sign take the host's fp32 mean|theta|) gives the same delta' rows, bit for bit, as the host vector
    of nets.py:108-112 passed through nicnes_set_mutation('scale'); the Mutator takes this path."""
    import nicnes
    from nicnes import mutations as MU
    dims = O.Dims()
    theta = O.make_theta(dims, 4, 4.0, 0.1)
    theta[:dims.E * dims.F:7] = 0.0
    theta[1:dims.E * dims.F:11] = -0.0
    table = O.noise_table(NOISE_LEN, 123)
    e = nicnes.Engine(max_batch=8, max_members=3, noise_len=NOISE_LEN, noise_seed=SEED)
    try:
        e.set_noise_table(table)
        e.set_theta(theta)
        e.set_mutation('scale', MU.proportional_vector(theta))
        want = e.noise_vectors(IT, 0, 3, SIGMA).cpu().numpy()
        e.set_mutation('plain')
        e.set_mutation_proportional(float(MU.proportional_mean(e.theta()[1])))
        got = e.noise_vectors(IT, 0, 3, SIGMA).cpu().numpy()
        assert np.array_equal(got, want)
        assert e.mutation_mode == 2
        assert e.theta_zeros() == int((theta == 0).sum()) > 0
        with pytest.raises(nicnes.NicnesError):
            e.set_mutation_proportional(float('nan'))
    finally:
        e.close()
