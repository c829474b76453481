"""CIDEr-D, restated in pure Python -- TEST INFRASTRUCTURE ONLY (oracle/).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module.

The reference scores captions with ``pyciderevalcap.ciderD.ciderD.CiderD(df='coco-train-idxs')``
(/root/reference/src/captioning/policies.py:18-19,72,180). That code lives in the git submodule
``cider`` -> git@github.com:rubencart/cider.git (/root/reference/.gitmodules:1-3), a fork of
vrama91/cider via ruotianluo/cider; the pinned commit is unknown and the directory is empty in
/root/reference, so it cannot be imported. This file restates the published CIDEr-D algorithm of
that lineage, in the same iteration order the upstream dict code uses:

  precook        n-gram counts for n = 1..4 of ``s.split()``
  counts2vec     vec[n][g] = tf * (ref_len - log(max(1, df[g]))); norm[n] = sqrt(sum vec^2);
                 length = number of BIGRAMS (upstream ``if n == 1: length += term_freq`` quirk)
  sim            sum_g min(vh[g], vr[g]) * vr[g], / (|vh||vr|) when both non-zero,
                 * e**(-(len_h - len_r)**2 / (2 sigma^2)), sigma = 6
  score          mean_n(sum_refs sim) / n_refs * 10
  fixed-df mode  document_frequency from a table, ref_len = log(raw ref_len)

The hypothesis / reference strings are built like the reference does
(``array_to_str``, /root/reference/src/algorithm/tools/utils.py:34-40: decimal ids separated by
spaces, up to and including the first 0) and the per-row gts mapping ``gts[i // seq_per_img]``
(/root/reference/src/captioning/policies.py:160-178).

Parity status: UNPINNED against the reference implementation (absent submodule); pinned by the
known-answer tests in tests/test_cider_oracle.py.
"""
from collections import defaultdict
import math

import numpy as np


def array_to_str(arr):
    """/root/reference/src/algorithm/tools/utils.py:34-40"""
    out = ''
    for i in range(len(arr)):
        out += str(int(arr[i])) + ' '
        if arr[i] == 0:
            break
    return out.strip()


def precook(s, n=4):
    words = s.split()
    counts = defaultdict(int)
    for k in range(1, n + 1):
        for i in range(len(words) - k + 1):
            counts[tuple(words[i:i + k])] += 1
    return counts


class CiderDOracle:
    """Fixed-df CIDEr-D (the ``df='coco-train-idxs'`` mode of the reference)."""

    def __init__(self, document_frequency, ref_len_raw, n=4, sigma=6.0):
        self.n = n
        self.sigma = sigma
        # n-grams are tuples of word strings; accept integer-id tuples too
        self.document_frequency = defaultdict(
            float, {tuple(str(w) for w in g): float(v) for g, v in document_frequency.items()})
        self.ref_len = np.log(float(ref_len_raw))

    def counts2vec(self, cnts):
        vec = [defaultdict(float) for _ in range(self.n)]
        length = 0
        norm = [0.0 for _ in range(self.n)]
        for (ngram, term_freq) in cnts.items():
            df = np.log(max(1.0, self.document_frequency[ngram]))
            n = len(ngram) - 1
            vec[n][ngram] = float(term_freq) * (self.ref_len - df)
            norm[n] += pow(vec[n][ngram], 2)
            if n == 1:
                length += term_freq
        norm = [np.sqrt(x) for x in norm]
        return vec, norm, length

    def sim(self, vec_hyp, vec_ref, norm_hyp, norm_ref, length_hyp, length_ref):
        delta = float(length_hyp - length_ref)
        val = np.array([0.0 for _ in range(self.n)])
        for n in range(self.n):
            for (ngram, count) in vec_hyp[n].items():
                val[n] += min(vec_hyp[n][ngram], vec_ref[n][ngram]) * vec_ref[n][ngram]
            if (norm_hyp[n] != 0) and (norm_ref[n] != 0):
                val[n] /= (norm_hyp[n] * norm_ref[n])
            assert not math.isnan(val[n])
            val[n] *= np.e ** (-(delta ** 2) / (2 * self.sigma ** 2))
        return val

    def score_one(self, hyp, refs):
        vec, norm, length = self.counts2vec(precook(hyp, self.n))
        score = np.array([0.0 for _ in range(self.n)])
        for ref in refs:
            vec_ref, norm_ref, length_ref = self.counts2vec(precook(ref, self.n))
            score += self.sim(vec, vec_ref, norm, norm_ref, length, length_ref)
        score_avg = np.mean(score)
        score_avg /= len(refs)
        score_avg *= 10.0
        return score_avg

    def compute_score(self, gts, res):
        """Same calling convention as CiderD.compute_score: gts {id: [ref strs]},
        res [{'image_id': id, 'caption': [hyp str]}] -> (mean, np.array(scores))."""
        scores = []
        for r in res:
            hypo = r['caption']
            ref = gts[r['image_id']]
            assert type(hypo) is list and len(hypo) == 1
            assert type(ref) is list and len(ref) > 0
            scores.append(self.score_one(hypo[0], ref))
        return np.mean(np.array(scores)), np.array(scores)


def rollout_fitness(scorer, seq, gts_rows, seq_per_img=1):
    """CaptPolicy.rollout for fitness 'greedy' (/root/reference/src/captioning/policies.py:86-128,
    145-193): 100 * mean CIDEr-D over the decoded rows. ``seq`` int [N, 16]; ``gts_rows`` is the
    per-image list of int arrays [n_i, 16] (data['gts'])."""
    batch_size = seq.shape[0]
    res = [{'image_id': i, 'caption': [array_to_str(seq[i])]} for i in range(batch_size)]
    gts_img = [[array_to_str(g[j]) for j in range(len(g))] for g in gts_rows]
    gts = {i: gts_img[i % batch_size // seq_per_img] for i in range(batch_size)}
    score, scores = scorer.compute_score(gts, res)
    return float(score * 100), scores


# greedy_* fitness criteria (pinned by tests/golden/fitness_criteria.npz, made from the reference's own
# classes by scripts/make_golden.py). Codes match nicnes_set_fitness_mode.
CRITERIA = {'greedy': 0, 'greedy_logprob': 1, 'greedy_expprob': 2, 'greedy_linprob': 3, 'greedy_avgprob': 4,
            'sample': 5, 'self_critical': 6, 'sc_loss': 7}


def criterion_fitness(mode, lp, seq, scores):
    """``crit(sample_logprobs, gen_result, rewards)`` of CaptPolicy.rollout (policies.py:119-123) for
    the criteria Fitness.get_criterium picks (policies.py:50-61): AltLog (fitness.py:43-64), Exp
    (:90-109), Lin (:112-132), AvgLog (:67-86), and Log (:12-40) for sc_loss. Elementwise in fp32 like torch; the sums in fp64.
    ``lp`` f32 [N, T] per-step log-prob of the chosen token, ``seq`` [N, T], ``scores`` [N] CIDEr-D
    per row (rewards = scores repeated over T, policies.py:191; cast to fp32 at policies.py:121)."""
    code = CRITERIA[mode] if isinstance(mode, str) else int(mode)
    lp = np.asarray(lp, np.float32)
    N, T = lp.shape
    reward = np.repeat(np.asarray(scores, np.float64).astype(np.float32)[:, None], T, 1)
    mask = np.concatenate([np.ones((N, 1), np.float32), (np.asarray(seq)[:, :-1] > 0).astype(np.float32)], 1)
    p = np.exp(lp)
    pfact = np.log10(p + np.float32(1 / 9)) + np.float32(np.log10(9))
    if code == 1:
        out = pfact * reward * mask
    elif code == 2:
        out = (np.exp(p) - np.float32(1)) / np.float32(math.e - 1) * reward * mask
    elif code == 3:
        out = p * reward * mask
    elif code == 4:
        out = np.float32(0.5) * reward * mask + np.float32(0.5) * pfact * reward * mask
    elif code == 7:                     # sc_loss: LogFitnessCriterion (fitness.py:12-40), rewards = sample - greedy
        out = -lp * reward * mask
    else:
        raise ValueError('criterion %r' % (mode,))
    return float(out.astype(np.float64).sum() / mask.astype(np.float64).sum())


def document_frequency_from_refs(ref_sets):
    """df as self-critical's prepro_ngrams builds it: for every image (a set of ref strings),
    each distinct n-gram over its refs counts once. Returns (dict, ref_len_raw=len(ref_sets))."""
    df = defaultdict(float)
    for refs in ref_sets:
        grams = set()
        for r in refs:
            grams.update(precook(r).keys())
        for g in grams:
            df[g] += 1
    return dict(df), len(ref_sets)
