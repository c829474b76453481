"""GPU parity: the HIP path through the C ABI against the CPU oracle (oracle/) on the same seeded
inputs. Tokens, noise indices, ranks and the weighted noise sum are compared bit-exactly; CIDEr-D
fitness (fp64, different reduction order) to 1e-9 relative; Adam bit-exactly against the
reference-generated golden fixture."""
import numpy as np
import pytest

torch = pytest.importorskip('torch')

pytestmark = pytest.mark.gpu

from oracle import oracle as O          # noqa: E402
from oracle import cider_ref as CR      # noqa: E402

NOISE_LEN = 1 << 23
SIGMA = 0.01


@pytest.fixture(scope='module')
def eng():
    import nicnes
    assert torch.cuda.is_available(), 'GPU tests need a GPU'
    e = nicnes.Engine(max_batch=128, max_members=8, noise_len=NOISE_LEN, noise_seed=7)
    table = O.noise_table(NOISE_LEN, 123)
    e.set_noise_table(table)
    e._table_np = table
    yield e
    e.close()


def _load(eng, theta, fc, gts=None, df=None, ref_len_raw=4096):
    eng.set_theta(theta)
    if gts is None:
        gts = [np.zeros((1, 16), np.int32) for _ in range(fc.shape[0])]
    if df is None:
        df = {}
    import nicnes
    keys, vals = nicnes.df_table_arrays(df)
    eng.set_df_table(keys, vals, np.log(float(ref_len_raw)))
    eng.set_batch(fc, gts)


def _oracle_member(theta, table, idx, fc, dims):
    out = []
    for sign in (+1, -1):
        seq, lp, fr = O.decode(dims, O.perturb(theta, table, idx, SIGMA, sign), fc)
        out.append((seq, fr))
    return out


def _compare_tokens(gpu_seq, ora_seq, fragile):
    """bit-exact, except after a step the oracle marks fragile (lse-rounding-dependent tie)."""
    B, T = ora_seq.shape
    mism = 0
    for b in range(B):
        for t in range(T):
            if fragile[b, t]:
                break
            if gpu_seq[b, t] != ora_seq[b, t]:
                mism += 1
                break
    return mism


@pytest.mark.parametrize('gain,bias_std', [(4.0, 0.1), (1.0, 0.0)], ids=['wc', 'xavier'])
def test_decode_tokens_bit_exact(eng, gain, bias_std):
    dims = O.Dims()
    theta = O.make_theta(dims, 0, gain, bias_std)
    fc = np.random.Generator(np.random.PCG64(1234)).standard_normal((40, dims.F)).astype(np.float32)
    _load(eng, theta, fc)
    it, m0, cnt = 5, 3, 2
    _, seq = eng.evaluate(it, m0, cnt, SIGMA, return_seq=True)
    seq = seq.cpu().numpy()
    idx = eng.noise_indices(it, m0, cnt).cpu().numpy()
    for k in range(cnt):
        assert idx[k] == O.noise_index(7, it, m0 + k, NOISE_LEN, dims.D)
        for s, (oseq, fr) in enumerate(_oracle_member(theta, eng._table_np, int(idx[k]), fc, dims)):
            assert _compare_tokens(seq[k, s], oseq, fr) == 0, (k, s, seq[k, s][:3], oseq[:3])


def test_decode_tiny_batch_and_slabs(eng):
    """B not a multiple of 32 and B > 128 (two row slabs) decode the same rows identically."""
    dims = O.Dims()
    theta = O.make_theta(dims, 3, 4.0, 0.1)
    fc = np.random.Generator(np.random.PCG64(99)).standard_normal((5, dims.F)).astype(np.float32)
    _load(eng, theta, fc)
    _, seq5 = eng.evaluate(1, 0, 1, SIGMA, return_seq=True)
    idx = int(eng.noise_indices(1, 0, 1).cpu().numpy()[0])
    for s, (oseq, fr) in enumerate(_oracle_member(theta, eng._table_np, idx, fc, dims)):
        assert _compare_tokens(seq5.cpu().numpy()[0, s], oseq, fr) == 0


@pytest.mark.parametrize('n_refs', [5, 10], ids=['image_tables', 'scan_over_8_refs'])
def test_cider_fitness_matches_oracle(eng, n_refs):
    """5 refs per image: the per-image n-gram table kernel; 10 (> IMG_MAXR): the per-reference scan."""
    import nicnes.synthetic as S
    dims = O.Dims()
    theta = O.make_theta(dims, 0, 4.0, 0.1)
    B = 24
    fc = np.random.Generator(np.random.PCG64(1234)).standard_normal((B, dims.F)).astype(np.float32)
    # references derived from the oracle's own base caption
    base, _, _ = O.decode(dims, theta, fc)
    gts, df, ref_len_raw = S.build_references(base, dims.vocab_size, seed=11, n_refs=n_refs, df_sets=256)
    _load(eng, theta, fc, gts, df, ref_len_raw)
    fit, seq = eng.evaluate(2, 0, 3, SIGMA, return_seq=True)
    fit, seq = fit.cpu().numpy(), seq.cpu().numpy()
    scorer = CR.CiderDOracle(df, ref_len_raw)
    for k in range(3):
        for s in range(2):
            f_ref, _ = CR.rollout_fitness(scorer, seq[k, s], gts)
            assert abs(fit[k, s] - f_ref) <= 1e-9 * max(1.0, abs(f_ref)), (k, s, fit[k, s], f_ref)
    assert fit.max() > 0.0


def _mask(seq):
    """positions the criteria count: t = 0, then seq[t-1] > 0 (src/captioning/fitness.py:57-58)"""
    return np.concatenate([np.ones((seq.shape[0], 1), bool), seq[:, :-1] > 0], 1)


def test_logprobs_match_oracle(eng):
    """seq_logprobs (nets.py:208,241): the greedy token's log-prob, -lse of the step, on every
    position a criterion counts; 1e-5 absolute (lse summed in another order than the oracle's)."""
    dims = O.Dims()
    theta = O.make_theta(dims, 0, 4.0, 0.1)
    fc = np.random.Generator(np.random.PCG64(4321)).standard_normal((36, dims.F)).astype(np.float32)
    _load(eng, theta, fc)
    _, seq, lp = eng.evaluate(3, 0, 2, SIGMA, return_seq=True, return_lp=True)
    seq, lp = seq.cpu().numpy(), lp.cpu().numpy()
    idx = eng.noise_indices(3, 0, 2).cpu().numpy()
    for k in range(2):
        for s, sign in enumerate((+1, -1)):
            oseq, olp, fr = O.decode(dims, O.perturb(theta, eng._table_np, int(idx[k]), SIGMA, sign), fc)
            assert np.array_equal(seq[k, s], oseq)
            m = _mask(oseq)
            assert np.abs(lp[k, s][m] - olp[m]).max() <= 1e-5
            assert (lp[k, s][m] <= 0).all() and np.isfinite(lp[k, s]).all()


@pytest.mark.parametrize('n_refs', [5, 10], ids=['image_tables', 'scan_over_8_refs'])
@pytest.mark.parametrize('mode', ['greedy_logprob', 'greedy_expprob', 'greedy_linprob', 'greedy_avgprob'])
def test_fitness_criteria_match_oracle(eng, mode, n_refs):
    """greedy_* fitness (policies.py:50-61,119-123; fitness.py:43-132) on the GPU against the oracle
    criterion (pinned by tests/golden/fitness_criteria.npz): 1e-6 relative on the GPU's own log-probs,
    1e-5 relative end to end against the oracle's decode."""
    import nicnes.synthetic as S
    dims = O.Dims()
    theta = O.make_theta(dims, 0, 4.0, 0.1)
    B = 24
    fc = np.random.Generator(np.random.PCG64(1234)).standard_normal((B, dims.F)).astype(np.float32)
    base, _, _ = O.decode(dims, theta, fc)
    gts, df, ref_len_raw = S.build_references(base, dims.vocab_size, seed=11, n_refs=n_refs, df_sets=256)
    _load(eng, theta, fc, gts, df, ref_len_raw)
    eng.set_fitness_mode(mode)
    try:
        fit, seq, lp = eng.evaluate(2, 0, 2, SIGMA, return_seq=True, return_lp=True)
        fit_nolp = eng.evaluate(2, 0, 2, SIGMA).cpu().numpy()
    finally:
        eng.set_fitness_mode('greedy')
    fit, seq, lp = fit.cpu().numpy(), seq.cpu().numpy(), lp.cpu().numpy()
    assert np.array_equal(fit, fit_nolp)                  # internal log-prob buffer == caller's
    scorer = CR.CiderDOracle(df, ref_len_raw)
    idx = eng.noise_indices(2, 0, 2).cpu().numpy()
    for k in range(2):
        for s, sign in enumerate((+1, -1)):
            _, scores = CR.rollout_fitness(scorer, seq[k, s], gts)
            f_own = CR.criterion_fitness(mode, lp[k, s], seq[k, s], scores)
            assert abs(fit[k, s] - f_own) <= 1e-6 * max(1.0, abs(f_own)), (k, s, fit[k, s], f_own)
            oseq, olp, _ = O.decode(dims, O.perturb(theta, eng._table_np, int(idx[k]), SIGMA, sign), fc)
            assert np.array_equal(seq[k, s], oseq)
            f_ora = CR.criterion_fitness(mode, olp, oseq, scores)
            assert abs(fit[k, s] - f_ora) <= 1e-5 * max(1.0, abs(f_ora)), (k, s, fit[k, s], f_ora)
    assert fit.max() > 0.0


def test_set_batch_rejects_images_without_references(eng):
    """CiderD asserts len(ref) > 0 for every image (upstream cider_scorer); the engine refuses such a
    batch with a status instead of scoring a 0/0, and a good batch loads again afterwards."""
    import nicnes
    dims = O.Dims()
    fc = np.random.Generator(np.random.PCG64(5)).standard_normal((4, dims.F)).astype(np.float32)
    gts = [np.ones((2, 16), np.int32), np.zeros((0, 16), np.int32), np.ones((1, 16), np.int32),
           np.ones((3, 16), np.int32)]
    eng.set_theta(O.make_theta(dims, 0, 4.0, 0.1))
    with pytest.raises(nicnes.NicnesError):
        eng.set_batch(fc, gts)
    with pytest.raises(nicnes.NicnesError):
        eng.evaluate(1, 0, 1, SIGMA)                       # no batch loaded
    with pytest.raises(ValueError):
        eng.set_batch(fc, gts[:3])
    gts[1] = np.ones((1, 16), np.int32)
    eng.set_batch(fc, gts)
    assert np.isfinite(eng.evaluate(1, 0, 1, SIGMA).cpu().numpy()).all()


def test_fitness_mode_rejects_unsupported(eng):
    import nicnes
    for bad in ('beam', 8, -1):
        with pytest.raises((nicnes.NicnesError, ValueError, RuntimeError)):
            eng.set_fitness_mode(bad)
    eng.set_fitness_mode('greedy')


def test_rank_weights_bit_exact(eng):
    rng = np.random.default_rng(5)
    fit = np.round(rng.random((300, 2)) * 20) / 2.0        # many ties
    cr, w = eng.rank_weights(torch.from_numpy(fit).cuda())
    w_ref, cr_ref = O.weights_from_fitness(fit)
    assert np.array_equal(cr.cpu().numpy(), cr_ref)
    assert np.array_equal(w.cpu().numpy(), w_ref)


def test_rank_docstring_known_answer(eng, golden_dir):
    z = np.load(golden_dir + '/ranks.npz')
    cr, _ = eng.rank_weights(torch.from_numpy(z['x']).cuda())
    assert np.allclose(cr.cpu().numpy(), z['y'], atol=1e-8)


def test_grad_bit_exact(eng):
    dims = O.Dims()
    P, it = 6, 9
    rng = np.random.default_rng(1)
    fit = rng.random((P, 2))
    w_ref, _ = O.weights_from_fitness(fit)
    w = torch.from_numpy(w_ref).cuda()
    g = eng.grad_partial(it, 0, P, w, SIGMA).cpu().numpy()
    idx = [O.noise_index(7, it, i, NOISE_LEN, dims.D) for i in range(P)]
    g_ref = O.gradient(fit, eng._table_np, idx, SIGMA, dims.D) * np.float32(2 * P)   # unscaled sum
    acc = np.zeros(dims.D, np.float64)
    for i in range(P):
        acc += np.float64(w_ref[i]) * (np.float32(SIGMA) * eng._table_np[idx[i]: idx[i] + dims.D]).astype(np.float64)
    assert np.array_equal(g, acc.astype(np.float32))
    assert np.allclose(g, g_ref, rtol=1e-6, atol=1e-9)


def test_adam_matches_reference_golden(golden_dir):
    """Adam on the engine vs the imported reference Adam (tests/golden/adam.npz): the engine is
    created with a D-sized theta only through its public API, so use the full dims and embed the
    1000-long fixture at the front of theta with zero gradient elsewhere."""
    import nicnes
    z = np.load(golden_dir + '/adam.npz')
    e = nicnes.Engine(max_batch=8, max_members=1, noise_len=1 << 22)
    try:
        D = e.D
        n = z['theta0'].size
        theta = np.zeros(D, np.float32)
        theta[:n] = z['theta0']
        e.set_theta(theta)                      # fp32 origin: reference first-step semantics
        for k in range(3):
            gsum = np.zeros(D, np.float32)
            # the engine computes g = gsum / (2P); feed gsum = g * 2 with P = 1 (exact: power of 2)
            gsum[:n] = z['grads'][k] * np.float32(2.0)
            ratio = e.adam_step(torch.from_numpy(gsum).cuda(), 1, float(z['l2coeff']), float(z['stepsize']))
            t64, _ = e.theta()
            assert np.array_equal(t64.cpu().numpy()[:n], z['thetas'][k]), k
            m, v, t = e.adam_state()
            assert np.array_equal(m.cpu().numpy()[:n], z['ms'][k]) and np.array_equal(v.cpu().numpy()[:n], z['vs'][k])
            assert t == k + 1
            assert ratio > 0
    finally:
        e.close()


def _embed(e, arr, dtype):
    out = np.zeros(e.D, dtype)
    out[:arr.size] = arr
    return out


def test_sgd_matches_reference_golden(golden_dir):
    """Fused SGD form vs the imported reference SGD driven like run_master (tests/golden/sgd.npz)."""
    import nicnes
    z = np.load(golden_dir + '/sgd.npz')
    e = nicnes.Engine(max_batch=8, max_members=1, noise_len=1 << 22)
    try:
        n = z['theta0'].size
        e.set_theta(_embed(e, z['theta0'], np.float32))
        for k in range(3):
            gsum = _embed(e, z['grads'][k] * np.float32(2.0), np.float32)
            ratio = e.sgd_step(torch.from_numpy(gsum).cuda(), 1, float(z['l2coeff']), float(z['stepsize']),
                               float(z['momentum']))
            t64, t32 = e.theta()
            assert np.array_equal(t64.cpu().numpy()[:n], z['thetas'][k]), k
            assert np.array_equal(t32.cpu().numpy()[:n], z['thetas'][k].astype(np.float32))
            _, v, t = e.adam_state()
            assert np.array_equal(v.cpu().numpy()[:n], z['vs'][k]) and t == k + 1
            assert ratio > 0
    finally:
        e.close()


def test_optimizer_update_globalg_forms(golden_dir):
    """Optimizer.update(globalg): fp32 globalg on the first step (adam.npz, host-side -g + l2*theta)
    and fp64 globalg from the first step (adam_globalg64.npz)."""
    import nicnes
    e = nicnes.Engine(max_batch=8, max_members=1, noise_len=1 << 22)
    try:
        z = np.load(golden_dir + '/adam.npz')
        n = z['theta0'].size
        e.set_theta(_embed(e, z['theta0'], np.float32))
        theta = z['theta0'].copy()
        for k in range(3):
            gg = -z['grads'][k] + float(z['l2coeff']) * theta       # fp32 at k=0, fp64 after (fact 8)
            e.optimizer_update(_embed(e, gg, gg.dtype), 'adam', stepsize=float(z['stepsize']))
            theta = e.theta()[0].cpu().numpy()[:n]
            assert np.array_equal(theta, z['thetas'][k]), k
        z = np.load(golden_dir + '/adam_globalg64.npz')
        n = z['theta0'].size
        e.set_theta(_embed(e, z['theta0'], np.float32))
        e.set_adam_state(np.zeros(e.D), np.zeros(e.D), 0)
        for k in range(2):
            e.optimizer_update(_embed(e, z['globalgs'][k], np.float64), 'adam', stepsize=float(z['stepsize']))
            assert np.array_equal(e.theta()[0].cpu().numpy()[:n], z['thetas'][k]), k
    finally:
        e.close()


def test_engine_worker_and_dispatched_master(eng):
    """EngineWorker.fitness_batch == Engine.evaluate; one dispatched iteration over the in-process
    transport gives the same theta as the local (PopulationRunner) loop."""
    import threading
    import nicnes.synthetic as S
    from nicnes import config as C, master as M, nes as N, transport as T
    dims = O.Dims()
    theta = O.make_theta(dims, 0, 4.0, 0.1)
    B, P = 16, 8
    fc = np.random.Generator(np.random.PCG64(1234)).standard_normal((B, dims.F)).astype(np.float32)
    base, _, _ = O.decode(dims, theta, fc)
    gts, df, ref_len_raw = S.build_references(base, dims.vocab_size, seed=11, df_sets=256)
    _load(eng, theta, fc, gts, df, ref_len_raw)
    exp = {'algorithm': 'nic_nes', 'nb_offspring': P,
           'config': {'noise_stdev': SIGMA, 'batch_size': B, 'l2coeff': 1e-7, 'snapshot_freq': 0},
           'policy_options': {'net': 'fc_caption', 'fitness': 'greedy', 'model_options': {}},
           'optimizer_options': {'type': 'adam', 'args': {'stepsize': 1e-3}}}
    spec = C.ExperimentSpec(exp)
    batch = {'fc_feats': fc, 'gts': gts}
    worker = N.EngineWorker(eng, spec, worker_id=0)
    res = worker.fitness_batch(0, N.NESTask(batch_data=batch, noise_stdev=SIGMA, iteration=4), 0, P)
    fit = eng.evaluate(4, 0, P, SIGMA).cpu().numpy()
    assert np.array_equal(np.stack([r.fitness for r in res]), fit)
    assert [r.noise_idx for r in res] == [O.noise_index(7, 4, m, NOISE_LEN, dims.D) for m in range(P)]

    eng.set_theta(theta)
    local = M.EngineMaster(spec, eng)
    local.run([batch], max_iterations=1)
    want = eng.theta()[0].cpu().numpy()

    eng.set_theta(theta)
    eng.set_adam_state(np.zeros(eng.D), np.zeros(eng.D), 0)
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        master = M.EngineMaster(spec, eng, log_dir=d)
        store = T.LocalStore()
        # worker and master share one engine here: the worker runs to completion before the master
        # updates (it only needs the task), so run it synchronously after the task is declared.
        mc = T.MasterClient(store)
        orig_declare = mc.declare_task

        def declare_and_work(task):
            tid = orig_declare(task)
            M.run_worker(T.WorkerClient(store), N.EngineWorker(eng, spec, worker_id=1), chunk=3, max_tasks=1)
            return tid
        mc.declare_task = declare_and_work
        master.run_dispatched(mc, [batch], max_iterations=1, result_timeout=60)
    assert np.array_equal(eng.theta()[0].cpu().numpy(), want)


def test_exact_tie_pass_matches_oracle(monkeypatch):
    """The exact second pass of the greedy tie rule (normally taken only when more records than
    tracked fall in the log_softmax tie window) forced on every step: tokens still match."""
    import nicnes
    monkeypatch.setenv('NICNES_FORCE_EXACT', '1')
    e = nicnes.Engine(max_batch=64, max_members=2, noise_len=NOISE_LEN, noise_seed=7)
    try:
        table = O.noise_table(NOISE_LEN, 123)
        e.set_noise_table(table)
        dims = O.Dims()
        theta = O.make_theta(dims, 5, 4.0, 0.1)
        fc = np.random.Generator(np.random.PCG64(4321)).standard_normal((40, dims.F)).astype(np.float32)
        _load(e, theta, fc)
        _, seq = e.evaluate(3, 0, 1, SIGMA, return_seq=True)
        seq = seq.cpu().numpy()
        assert e.stats()['tie_fallbacks'] >= 16          # one per decode step of the workgroup
        idx = int(e.noise_indices(3, 0, 1).cpu().numpy()[0])
        for s, (oseq, fr) in enumerate(_oracle_member(theta, table, idx, fc, dims)):
            assert _compare_tokens(seq[0, s], oseq, fr) == 0
    finally:
        e.close()


@pytest.mark.parametrize('shape', [(1, 4), (4, 2)], ids=['fused', 'split_G2S4'])
def test_bounded_lse_undecided_rows_take_the_exact_pass(monkeypatch, shape):
    """Greedy-only decodes bound lse from an exp-sum over pair maxima; a record whose window state the
    bound leaves open goes to the exact pass. NICNES_LSE_MARGIN=1e5 widens the bound so that rows with
    a record within ~0.004 of the max are undecided: the exact pass must run and the tokens still match the oracle."""
    import nicnes
    monkeypatch.setenv('NICNES_LSE_MARGIN', '1e5')
    e = nicnes.Engine(max_batch=64, max_members=2, noise_len=NOISE_LEN, noise_seed=7)
    try:
        table = O.noise_table(NOISE_LEN, 123)
        e.set_noise_table(table)
        dims = O.Dims()
        theta = O.make_theta(dims, 0, 1.0, 0.0)             # xavier: near-uniform logits, many near ties
        fc = np.random.Generator(np.random.PCG64(99)).standard_normal((40, dims.F)).astype(np.float32)
        _load(e, theta, fc)
        e.set_decode_split(*shape)
        _, seq = e.evaluate(3, 0, 2, SIGMA, return_seq=True)
        seq = seq.cpu().numpy()
        assert e.stats()['tie_fallbacks'] > 0
        for k in range(2):
            idx = int(e.noise_indices(3, k, 1).cpu().numpy()[0])
            for s, (oseq, fr) in enumerate(_oracle_member(theta, table, idx, fc, dims)):
                assert _compare_tokens(seq[k, s], oseq, fr) == 0
    finally:
        e.close()


@pytest.mark.parametrize('P', [2048, 8192, 1000, 1024, 1025, 64, 1],
                         ids=['P2048', 'P8192', 'P1000', 'P1024_small_max', 'P1025_sort', 'P64', 'P1'])
def test_rank_weights_bit_exact_large(eng, P):
    """Both rank paths: the one-launch count (2P <= 2048 entries: the bench's P = 512 and its 64 / 128 per GPU)
    and the sort-based rank (chunk bitonic sort + lower bounds) at configs[3]'s pop=2048 and beyond; the boundary
    on either side; many ties, -0.0 / +0.0 and NaN (last, as numpy's argsort places it)."""
    rng = np.random.default_rng(P)
    fit = np.round(rng.random((P, 2)) * 200) / 4.0
    if P >= 8:
        fit[3, 0], fit[5, 1], fit[7, 0] = -0.0, 0.0, np.nan
    cr, w = eng.rank_weights(torch.from_numpy(fit).cuda())
    w_ref, cr_ref = O.weights_from_fitness(fit)
    assert np.array_equal(cr.cpu().numpy(), cr_ref)
    assert np.array_equal(w.cpu().numpy(), w_ref)
