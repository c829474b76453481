"""Synthetic fc_caption workloads -- the data/checkpoints of the reference are not
available offline, so every run uses seeded synthetic inputs of the reference's shapes:

  fc        N(0,1) fp32 [B, 2048] (seed 1234); 'bu' variant ReLU(N(0,1)) (seed 1235)
  theta     FCModel init of PolicyNet.initialize_params (/root/reference/src/algorithm/nets.py:62-69):
            xavier_normal_ weights, zero biases, drawn from numpy PCG64(seed)
  refs      5 per image, length L ~ U[8, 16], from the base-theta greedy caption with 30 % token
            substitution, ending with 0 when L < 16 (a zero-padded label row)
  df table  document frequency over 4096 synthetic reference sets (the batch's + generated ones),
            ref_len = log(4096) -- the fixed-df mode of CiderD(df='coco-train-idxs')
  noise     2^27-entry fp32 Gaussian table, numpy PCG64(123)
"""
from collections import defaultdict

import numpy as np

from .engine import df_table_arrays


class Dims:
    def __init__(self, vocab_size=9487, E=128, R=128, F=2048, T=16):
        self.vocab_size, self.V1, self.E, self.R, self.F, self.T = vocab_size, vocab_size + 1, E, R, F, T

    def shapes(self):
        V1, E, R, F = self.V1, self.E, self.R, self.F
        return [('img_embed.weight', (E, F)), ('img_embed.bias', (E,)), ('embed.weight', (V1, E)),
                ('logit.weight', (V1, R)), ('logit.bias', (V1,)), ('core.i2h.weight', (5 * R, E)),
                ('core.i2h.bias', (5 * R,)), ('core.h2h.weight', (5 * R, R)), ('core.h2h.bias', (5 * R,))]

    @property
    def D(self):
        return sum(int(np.prod(s)) for _, s in self.shapes())


def init_theta(dims, seed=0, gain=1.0, bias_std=0.0):
    """Flat fp32 theta in module registration order (nets.py:150-153, LSTMCore :81-82)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    parts = []
    for name, shp in dims.shapes():
        if name.endswith('weight'):
            std = gain * np.sqrt(2.0 / float(shp[1] + shp[0]))
            parts.append((rng.standard_normal(shp) * std).astype(np.float32).ravel())
        elif bias_std > 0:
            parts.append((rng.standard_normal(shp) * bias_std).astype(np.float32).ravel())
        else:
            parts.append(np.zeros(int(np.prod(shp)), np.float32))
    return np.concatenate(parts)


def fc_feats(B, F=2048, seed=1234, bu=False):
    x = np.random.Generator(np.random.PCG64(seed)).standard_normal((B, F)).astype(np.float32)
    return np.maximum(x, 0.0).astype(np.float32) if bu else x


def noise_table(n=1 << 27, seed=123):
    return np.random.Generator(np.random.PCG64(seed)).standard_normal(n, dtype=np.float32)


def substituted_refs(base_caption, vocab_size, rng, n_refs=5, T=16, p_sub=0.3):
    """n_refs zero-padded label rows derived from one caption."""
    base = [int(t) for t in base_caption if t > 0] or [1]
    rows = np.zeros((n_refs, T), np.int32)
    for j in range(n_refs):
        L = int(rng.integers(8, T + 1))
        toks = [base[k % len(base)] for k in range(L)]
        for k in range(L):
            if rng.random() < p_sub:
                toks[k] = int(rng.integers(1, vocab_size + 1))
        if L < T:
            toks[L - 1] = 0                       # the caption ends with the 0 token
        rows[j, :L] = toks
    return rows


def _row_ngrams(row, T=16):
    words = []
    for t in row[:T]:
        words.append(int(t))
        if t == 0:
            break
    out = set()
    for n in range(1, 5):
        for i in range(len(words) - n + 1):
            out.add(tuple(words[i:i + n]))
    return out


def build_references(base_captions, vocab_size, seed=4321, n_refs=5, df_sets=4096, T=16):
    """-> (gts: list of [n_refs, T] int32, df dict {ngram tuple: count}, ref_len_raw)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    gts = [substituted_refs(c, vocab_size, rng, n_refs, T) for c in base_captions]
    df = defaultdict(float)
    sets = list(gts)
    while len(sets) < df_sets:
        c = base_captions[int(rng.integers(0, len(base_captions)))]
        sets.append(substituted_refs(c, vocab_size, rng, n_refs, T))
    for refs in sets:
        grams = set()
        for r in refs:
            grams |= _row_ngrams(r, T)
        for g in grams:
            df[g] += 1.0
    return gts, dict(df), len(sets)


def setup_engine_workload(engine, B=128, theta_seed=0, fc_seed=1234, bu=False, noise=None, ref_seed=4321,
                          df_sets=4096, batches=1, theta_gain=1.0, bias_std=0.0):
    """Load a full synthetic workload into an Engine: noise table, theta, fc, refs + df.
    batches > 1: that many batches of B images each (per-member batches, single_batch: false), held
    with set_batches; fc / gts / base then cover all batches * B images in batch order.
    Returns dict(theta32, fc, gts, df, ref_len_raw, base)."""
    dims = Dims(engine.cfg.vocab_size, engine.cfg.input_encoding_size, engine.cfg.rnn_size,
                engine.cfg.fc_feat_size, engine.cfg.seq_length)
    if noise is None:
        noise = noise_table(engine.cfg.noise_len)
    engine.set_noise_table(noise)
    theta = init_theta(dims, theta_seed, theta_gain, bias_std)
    engine.set_theta(theta)
    n = B * batches
    fc = fc_feats(n, dims.F, fc_seed, bu)
    # the base-theta greedy captions seed the references: decode once with sigma = 0
    placeholder = [np.zeros((1, dims.T), np.int32) for _ in range(B)]
    engine.set_df_table(np.zeros(0, np.uint64), np.zeros(0), np.log(float(df_sets)))
    bases = []
    for g in range(batches):
        engine.set_batch(fc[g * B:(g + 1) * B], placeholder)
        _, seq = engine.evaluate(0, 0, 1, 0.0, return_seq=True)
        bases.append(seq[0, 0].cpu().numpy())
    base = np.concatenate(bases)
    gts, df, ref_len_raw = build_references(base, dims.vocab_size, ref_seed, 5, df_sets, dims.T)
    keys, vals = df_table_arrays(df)
    engine.set_df_table(keys, vals, np.log(float(ref_len_raw)))
    if batches == 1:
        engine.set_batch(fc, gts)
    else:
        engine.set_batches([(fc[g * B:(g + 1) * B], gts[g * B:(g + 1) * B]) for g in range(batches)])
    return dict(theta32=theta, fc=fc, gts=gts, df=df, ref_len_raw=ref_len_raw, base=base, dims=dims)
