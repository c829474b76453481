"""The HIP path against the REFERENCE itself at the benchmarked workload (no oracle in between):
tests/golden/decode_bench_xavier.npz and master_ranks_grad.npz hold FCModel._sample tokens and
NESMaster rank / gradient outputs that scripts/make_golden.py produced by importing the reference.

Workload = BASELINE.json configs[2] (pop=512, B=128, xavier theta seed 0, fc seed 1234, the 2^27
table, noise seed 0, iteration 1), configs[1]'s shape (pop=64, the split decode path) and
mscoco_nes.json's own batch_size 64 (decode_bench_b64.npz: the 64-row slab path) at both populations.
Bars: greedy tokens identical to the reference on every row end to end (>= 2,048 rows per shape, the
near-tie steps of the golden included: they are recorded); fitness of the engine
equal to the restated CIDEr-D of the reference's own tokens to 1e-9; centred ranks bit-exact; the
gradient within 1e-5 of max |g| (north_star). The measured agreement is written to
gpurun_out/reference_parity.json for DESIGN.md."""
import json
import os

import numpy as np
import pytest

torch = pytest.importorskip('torch')

pytestmark = pytest.mark.gpu

from oracle import cider_ref as CR      # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MARGIN = 1e-5
_report = {}


def _write_report():
    out = os.path.join(REPO, 'gpurun_out')
    os.makedirs(out, exist_ok=True)
    with open(os.path.join(out, 'reference_parity.json'), 'w') as f:
        json.dump(_report, f, indent=1)


@pytest.fixture(scope='module')
def goldens(golden_dir):
    return {n: np.load(golden_dir + '/%s.npz' % n) for n in ('decode_bench_xavier', 'decode_bench_b64')}


def _engine(P, golden):
    import nicnes
    import nicnes.synthetic as S
    assert torch.cuda.is_available(), 'GPU tests need a GPU'
    e = nicnes.Engine(max_batch=128, max_members=P, noise_len=int(golden['noise_len']),
                      noise_seed=int(golden['noise_seed']))
    wl = S.setup_engine_workload(e, B=int(golden['B']), noise=S.noise_table(int(golden['noise_len']),
                                                                            int(golden['table_seed'])))
    return e, wl


def _agree(seq, ref, margins):
    """(rows identical end to end, rows identical up to their first reference near-tie)"""
    full = int((seq == ref).all(axis=1).sum())
    upto = 0
    for b in range(ref.shape[0]):
        ok = True
        for t in range(ref.shape[1]):
            if margins[b, t] < MARGIN:
                break
            if seq[b, t] != ref[b, t]:
                ok = False
                break
        upto += ok
    return full, upto


@pytest.mark.parametrize('P, name', [(512, 'decode_bench_xavier'), (64, 'decode_bench_xavier'),
                                     (512, 'decode_bench_b64'), (64, 'decode_bench_b64')],
                         ids=['configs2_pop512_B128', 'configs1_pop64_B128', 'pop512_B64', 'pop64_B64'])
def test_tokens_and_fitness_match_reference(goldens, P, name):
    golden = goldens[name]
    e, wl = _engine(P, golden)
    try:
        ref = golden['seq'].astype(np.int32)
        mar = golden['margins']
        # the sigma = 0 decode that seeded the synthetic references is the reference's base decode
        full, upto = _agree(wl['base'], ref[0], mar[0])
        assert upto == ref.shape[1] and full == ref.shape[1]
        it, sigma = int(golden['iteration']), float(golden['sigma'])
        fit, seq = e.evaluate(it, 0, P, sigma, return_seq=True)
        fit, seq = fit.cpu().numpy(), seq.cpu().numpy()
        scorer = CR.CiderDOracle(wl['df'], wl['ref_len_raw'])
        rows = rows_full = rows_upto = 0
        fdiff = 0.0
        for k, mbr in enumerate(golden['members']):
            if mbr >= P:
                continue
            for s in range(2):
                r, m = ref[1 + 2 * k + s], mar[1 + 2 * k + s]
                full, upto = _agree(seq[mbr, s], r, m)
                rows += r.shape[0]
                rows_full += full
                rows_upto += upto
                f_ref = CR.rollout_fitness(scorer, r, wl['gts'])[0]
                fdiff = max(fdiff, abs(fit[mbr, s] - f_ref))
        assert rows >= (2048 if P == 512 or int(golden['B']) == 128 else 1024)
        assert rows_upto == rows and rows_full == rows
        assert fdiff <= 1e-9 * max(1.0, float(np.abs(fit).max()))
        _report['P%d_B%d' % (P, int(golden['B']))] = {
                              'decode_shape': list(e.decode_shape(int(golden['B']), P)), 'rows_compared': rows,
                              'rows_identical_end_to_end': rows_full, 'rows_identical_to_first_near_tie': rows_upto,
                              'near_tie_steps_in_golden': int((mar[1:] < MARGIN).sum()),
                              'max_abs_fitness_diff_vs_reference_tokens': fdiff}
        _write_report()
    finally:
        e.close()


@pytest.mark.parametrize('case, begin, count, path', [('c3', 1792, 256, 'fused'), ('c4', 448, 64, 'coop'),
                                                      ('c4', 0, 64, 'coop')],
                         ids=['configs3_rank7_of8', 'configs4_bu_rank7_of8', 'configs4_bu_rank0_of8'])
def test_rank_slices_match_reference(golden_dir, case, begin, count, path):
    """The exact per-GPU slice an 8-GPU run of configs[3] / configs[4] evaluates on one rank
    (evaluate(it, begin, count) with bench.py's member ranges), against FCModel._sample of the imported
    reference on the same members (tests/golden/decode_rank_slices.npz). configs[4] uses bottom-up ReLU
    features and runs on the coop path (64 members per GPU at B = 128, S = 4); configs[3] on the fused path."""
    import nicnes
    import nicnes.synthetic as S
    z = np.load(golden_dir + '/decode_rank_slices.npz')
    members = z[case + '_members']
    ref, mar = z[case + '_seq'].astype(np.int32), z[case + '_margins']
    e = nicnes.Engine(max_batch=128, max_members=count, noise_len=int(z['noise_len']),
                      noise_seed=int(z['noise_seed']))
    try:
        wl = S.setup_engine_workload(e, B=int(z['B']), fc_seed=int(z[case + '_fc_seed']), bu=bool(z[case + '_bu']),
                                     noise=S.noise_table(int(z['noise_len']), int(z['table_seed'])))
        full, upto = _agree(wl['base'], ref[0], mar[0])
        assert full == ref.shape[1], 'base-theta decode differs from the reference'
        assert e.decode_path(int(z['B']), count) == path
        fit, seq = e.evaluate(int(z['iteration']), begin, count, float(z['sigma']), return_seq=True)
        fit, seq = fit.cpu().numpy(), seq.cpu().numpy()
        scorer = CR.CiderDOracle(wl['df'], wl['ref_len_raw'])
        rows = rows_full = 0
        fdiff = 0.0
        for k, mbr in enumerate(members):
            if not begin <= mbr < begin + count:
                continue
            for s in range(2):
                r, m = ref[1 + 2 * k + s], mar[1 + 2 * k + s]
                full, upto = _agree(seq[mbr - begin, s], r, m)
                assert full == r.shape[0], (case, int(mbr), s, full)
                rows += r.shape[0]
                rows_full += full
                fdiff = max(fdiff, abs(fit[mbr - begin, s] - CR.rollout_fitness(scorer, r, wl['gts'])[0]))
        assert rows >= 4 * 2 * 128
        assert fdiff <= 1e-9 * max(1.0, float(np.abs(fit).max()))
        _report['%s_members_%d_%d' % (case, begin, begin + count)] = {
            'decode_path': path, 'decode_shape': list(e.decode_shape(int(z['B']), count)), 'rows_compared': rows,
            'rows_identical_end_to_end': rows_full, 'near_tie_steps_in_golden': int((mar[1:] < MARGIN).sum()),
            'max_abs_fitness_diff_vs_reference_tokens': fdiff}
        _write_report()
    finally:
        e.close()


def test_ranks_and_gradient_match_reference(golden_dir):
    import nicnes
    z = np.load(golden_dir + '/master_ranks_grad.npz')
    P = z['fit'].shape[0]
    e = nicnes.Engine(max_batch=8, max_members=P, noise_len=int(z['noise_len']), noise_seed=int(z['noise_seed']))
    try:
        import nicnes.synthetic as S
        e.set_noise_table(S.noise_table(int(z['noise_len']), 123))
        cr, w = e.rank_weights(torch.from_numpy(z['fit']).cuda())
        assert np.array_equal(cr.cpu().numpy(), z['cr'])
        cr_t, _ = e.rank_weights(torch.from_numpy(z['fit_ties']).cuda())
        x, a, b = z['fit_ties'].ravel(), cr_t.cpu().numpy().ravel(), z['cr_ties'].ravel()
        for v in np.unique(x):
            assert np.array_equal(np.sort(a[x == v]), np.sort(b[x == v])), v
        assert np.array_equal(e.noise_indices(int(z['iteration']), 0, P).cpu().numpy().astype(np.int64), z['idx'])
        gsum = e.grad_partial(int(z['iteration']), 0, P, w, float(z['sigma'])).cpu().numpy()
        g = gsum[z['J']] / np.float32(2 * P)
        err = float(np.abs(g - z['grad']).max() / np.abs(z['grad']).max())
        assert err <= 1e-5
        _report['master'] = {'P': int(P), 'ranks_bit_exact': True, 'grad_max_rel_err_vs_reference_fp32': err}
        _write_report()
    finally:
        e.close()
