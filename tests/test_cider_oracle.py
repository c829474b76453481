"""Known-answer tests of the restated CIDEr-D (oracle/cider_ref.py). The reference scorer lives in
the unvendored `cider` submodule, so these pin the restatement by hand-derived values
(parity with the reference implementation itself: unpinned)."""
import math
import os

import numpy as np
import pytest

from oracle import cider_ref as CR

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')


def test_array_to_str_includes_first_zero():
    # /root/reference/src/algorithm/tools/utils.py:34-40
    assert CR.array_to_str(np.array([5, 7, 0, 3, 0])) == '5 7 0'
    assert CR.array_to_str(np.array([0, 4])) == '0'
    assert CR.array_to_str(np.array([1, 2, 3])) == '1 2 3'


def test_identical_single_ref_scores_ten():
    s = CR.CiderDOracle({}, 10)            # empty df: every idf = log(10) > 0
    assert s.score_one('1 2 3 4 5', ['1 2 3 4 5']) == pytest.approx(10.0, rel=1e-12)


def test_disjoint_scores_zero():
    s = CR.CiderDOracle({}, 10)
    assert s.score_one('1 2 3', ['4 5 6']) == 0.0


def test_df_equal_ref_len_zeroes_the_ngram():
    # an n-gram seen in every reference set has idf = log(N) - log(N) = 0
    df = {('7',): 10.0}
    s = CR.CiderDOracle(df, 10)
    vec, norm, length = s.counts2vec(CR.precook('7 8'))
    assert vec[0][('7',)] == 0.0 and vec[0][('8',)] == pytest.approx(math.log(10))
    assert length == 1                      # one bigram: the 'length' is the bigram count


def test_length_penalty_uses_bigram_counts():
    s = CR.CiderDOracle({}, 100)
    hyp, ref = '1 2', '1 2 9 9 9 9 9'
    # unigrams/bigrams of hyp all in ref; delta = (1 - 6) bigrams
    sc = s.score_one(hyp, [ref])
    vh, nh, lh = s.counts2vec(CR.precook(hyp))
    vr, nr, lr = s.counts2vec(CR.precook(ref))
    assert (lh, lr) == (1, 6)
    pen = np.e ** (-(5.0 ** 2) / (2 * 36.0))
    val1 = sum(min(vh[0][g], vr[0][g]) * vr[0][g] for g in vh[0]) / (nh[0] * nr[0]) * pen
    val2 = sum(min(vh[1][g], vr[1][g]) * vr[1][g] for g in vh[1]) / (nh[1] * nr[1]) * pen
    assert sc == pytest.approx((val1 + val2) / 4 * 10, rel=1e-12)


def test_clipping_min_term():
    s = CR.CiderDOracle({}, 100)
    # hyp repeats a word more often than the ref: min(vh, vr) clips
    vh, nh, _ = s.counts2vec(CR.precook('3 3 3'))
    vr, nr, _ = s.counts2vec(CR.precook('3'))
    assert vh[0][('3',)] == pytest.approx(3 * math.log(100))
    sc = s.sim(vh, vr, nh, nr, 2, 0)
    assert sc[0] == pytest.approx(min(vh[0][('3',)], vr[0][('3',)]) * vr[0][('3',)] / (nh[0] * nr[0])
                                  * np.e ** (-4 / 72.0))


def test_rollout_fitness_dedup_equals_duplicated():
    """mean over 5x-duplicated rows == mean over unique rows (fixed df): the engine decodes
    unique images only."""
    rng = np.random.default_rng(3)
    B = 6
    seq = rng.integers(0, 20, (B, 16))
    gts = [rng.integers(1, 20, (5, 16)) for _ in range(B)]
    df, n = CR.document_frequency_from_refs([[CR.array_to_str(r) for r in g] for g in gts])
    s = CR.CiderDOracle(df, n)
    f_unique, _ = CR.rollout_fitness(s, seq, gts, 1)
    f_dup, _ = CR.rollout_fitness(s, np.repeat(seq, 5, axis=0), gts, 5)
    assert f_unique == pytest.approx(f_dup, rel=1e-12)


@pytest.mark.parametrize('mode', ['greedy_logprob', 'greedy_expprob', 'greedy_linprob', 'greedy_avgprob', 'sc_loss'])
def test_criterion_oracle_matches_reference_golden(mode):
    """greedy_* criteria (src/captioning/fitness.py:43-132) against the reference's own classes
    (tests/golden/fitness_criteria.npz, scripts/make_golden.py); the reference sums in fp32."""
    z = np.load(os.path.join(GOLDEN, 'fitness_criteria.npz'))
    for c in range(3):
        got = CR.criterion_fitness(mode, z['lp_%d' % c], z['seq_%d' % c], z['scores_%d' % c])
        ref = float(z['%s_%d' % (mode, c)])
        assert abs(got - ref) <= 1e-6 * max(1.0, abs(ref)), (c, got, ref)


def test_criterion_duplicate_rows_invariant():
    """The engine scores unique images once; the reference decodes each 5x (dataloader.py:175).
    The criterion is a ratio of sums, so 5 identical copies give the same value."""
    rng = np.random.Generator(np.random.PCG64(5))
    seq = rng.integers(0, 9, (6, 16))
    lp = -rng.exponential(1.0, (6, 16)).astype(np.float32)
    sc = rng.uniform(0, 2, 6)
    for mode in ('greedy_logprob', 'greedy_expprob', 'greedy_linprob', 'greedy_avgprob'):
        a = CR.criterion_fitness(mode, lp, seq, sc)
        b = CR.criterion_fitness(mode, np.repeat(lp, 5, 0), np.repeat(seq, 5, 0), np.repeat(sc, 5))
        assert abs(a - b) <= 1e-12 * max(1.0, abs(a))
