"""The reference CPU worker path, restated with torch-CPU ops -- TEST INFRASTRUCTURE ONLY.

Used by bench.py's cpu_baseline leg (kind "port") to time what one reference worker does per
population member, on the GPU box's host cores (the reference itself cannot travel there):

  NESWorker.fitness      /root/reference/src/algorithm/nic_nes/nic_nes_worker.py:115-161
    evolve theta+delta   /root/reference/src/algorithm/nets.py:101-114 (delta from the table here)
    rollout              /root/reference/src/captioning/policies.py:86-128
      FCModel._sample    /root/reference/src/captioning/nets.py:183-245 -- same torch ops: nn.Linear,
                         nn.Embedding, LSTMCore (:98-134), F.log_softmax, torch.max; 18 cell + 18 logit
                         steps; fc rows duplicated seq_per_img = 5 times (dataloader.py:175)
      compute_ciders     policies.py:145-193 with the pure-Python CIDEr-D of oracle/cider_ref.py
    theta - delta, rollout again
One single-threaded process per core, as src/main.py:8-11,144-153 runs workers; then the master leg
(time_master): NESMaster.gradient_estimate -- compute_centered_ranks, batched_weighted_sum in fp32
np.dot groups of 500 -- and Adam.update in fp64 numpy (nic_nes_master.py:123-137,170-221,
optimizers.py:15-22,78-83) over the P received noise vectors.
"""
import os
import time

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import cider_ref


class LSTMCoreRef(nn.Module):
    def __init__(self, E, R):
        super().__init__()
        self.rnn_size = R
        self.i2h = nn.Linear(E, 5 * R)
        self.h2h = nn.Linear(R, 5 * R)

    def forward(self, xt, state):
        all_input_sums = self.i2h(xt) + self.h2h(state[0][-1])
        sigmoid_chunk = torch.sigmoid(all_input_sums.narrow(1, 0, 3 * self.rnn_size))
        in_gate = sigmoid_chunk.narrow(1, 0, self.rnn_size)
        forget_gate = sigmoid_chunk.narrow(1, self.rnn_size, self.rnn_size)
        out_gate = sigmoid_chunk.narrow(1, self.rnn_size * 2, self.rnn_size)
        in_transform = torch.max(all_input_sums.narrow(1, 3 * self.rnn_size, self.rnn_size),
                                 all_input_sums.narrow(1, 4 * self.rnn_size, self.rnn_size))
        next_c = forget_gate * state[1][-1] + in_gate * in_transform
        next_h = out_gate * torch.tanh(next_c)
        return next_h, (next_h.unsqueeze(0), next_c.unsqueeze(0))


class FCModelRef(nn.Module):
    def __init__(self, vocab_size=9487, E=128, R=128, F_=2048, T=16):
        super().__init__()
        self.rnn_size, self.seq_length = R, T
        self.img_embed = nn.Linear(F_, E)
        self.embed = nn.Embedding(vocab_size + 1, E)
        self.logit = nn.Linear(R, vocab_size + 1)
        self.core = LSTMCoreRef(E, R)
        for p in self.parameters():
            p.requires_grad = False

    def sample(self, fc_feats):
        batch_size = fc_feats.size(0)
        z = fc_feats.new_zeros(1, batch_size, self.rnn_size)
        state = (z, z.clone())
        seq = fc_feats.new_zeros(batch_size, self.seq_length, dtype=torch.long)
        seq_logprobs = fc_feats.new_zeros(batch_size, self.seq_length)
        unfinished = None
        it = None
        for t in range(self.seq_length + 2):
            if t == 0:
                xt = self.img_embed(fc_feats)
            else:
                if t == 1:
                    it = fc_feats.new_zeros(batch_size, dtype=torch.long)
                xt = self.embed(it)
            output, state = self.core(xt, state)
            logprobs = F.log_softmax(self.logit(output), dim=1)
            if t == self.seq_length + 1:
                break
            sample_logprobs, it = torch.max(logprobs, 1)
            it = it.view(-1).long()
            if t >= 1:
                unfinished = (it > 0) if t == 1 else unfinished * (it > 0)
                it = it * unfinished.type_as(it)
                seq[:, t - 1] = it
                seq_logprobs[:, t - 1] = sample_logprobs.view(-1)
                if unfinished.sum() == 0:
                    break
        return seq, seq_logprobs


class RefWorker:
    """State of one reference worker process."""

    def __init__(self, theta32, fc_unique, gts, df, ref_len_raw, seq_per_img=5, vocab_size=9487):
        torch.set_num_threads(1)
        torch.set_grad_enabled(False)
        self.model = FCModelRef(vocab_size)
        self.theta = torch.from_numpy(np.ascontiguousarray(theta32))
        self.fc = torch.from_numpy(np.repeat(fc_unique, seq_per_img, axis=0))     # dataloader.py:175
        self.gts = gts
        self.seq_per_img = seq_per_img
        self.scorer = cider_ref.CiderDOracle(df, ref_len_raw)

    def rollout(self):
        seq, _ = self.model.sample(self.fc)
        fit, _ = cider_ref.rollout_fitness(self.scorer, seq.numpy(), self.gts, self.seq_per_img)
        return fit

    def fitness(self, delta32):
        delta = torch.from_numpy(delta32)
        nn.utils.vector_to_parameters(self.theta + delta, self.model.parameters())
        pos = self.rollout()
        nn.utils.vector_to_parameters(self.theta - delta, self.model.parameters())
        neg = self.rollout()
        return np.stack((pos, neg))


_W = None


def _init(args):
    global _W
    _W = RefWorker(*args)


def _member(delta32):
    t0 = time.perf_counter()
    f = _W.fitness(delta32)
    return f, time.perf_counter() - t0


def time_members(theta32, fc_unique, gts, df, ref_len_raw, deltas, processes):
    """Evaluate len(deltas) members on `processes` single-threaded worker processes (fork).
    Returns (members/s over the wall time, fitness array, per-member seconds)."""
    import multiprocessing as mp
    ctx = mp.get_context('fork')
    os.environ.setdefault('OMP_NUM_THREADS', '1')
    with ctx.Pool(processes, initializer=_init, initargs=((theta32, fc_unique, gts, df, ref_len_raw),)) as pool:
        pool.map(_noop, range(processes))                   # workers up (model built) before timing
        t0 = time.perf_counter()
        res = pool.map(_member, deltas, chunksize=1)
        wall = time.perf_counter() - t0
    fits = np.array([r[0] for r in res])
    secs = np.array([r[1] for r in res])
    return len(deltas) / wall, fits, secs


def _noop(_):
    return os.getpid()


def usable_cpus():
    """CPUs this process may run on: the cgroup v2 quota when one is set (a GPU box shares its host),
    else the affinity mask."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, 'sched_getaffinity') else (os.cpu_count() or 1)
    try:
        quota, period = open('/sys/fs/cgroup/cpu.max').read().split()[:2]
        if quota != 'max':
            n = min(n, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return n


def _centered_ranks(x):
    """compute_centered_ranks / compute_ranks (nic_nes_master.py:184-205): default argsort as the
    reference calls it"""
    r = np.empty(x.size, dtype=int)
    r[x.ravel().argsort()] = np.arange(x.size)
    y = r.reshape(x.shape).astype(np.float64)
    y /= (x.size - 1)
    y -= .5
    return y


def time_master(fitness, table, indices, sigma, theta32, l2coeff=1e-7, stepsize=1e-3):
    """The reference master's per-iteration leg over P results, timed: ranks, the fp32 weighted sum
    of the P noise vectors in groups of 500 (batched_weighted_sum), /2F, then Adam in fp64 numpy.
    The noise vectors are materialised first, as the master holds the received arrays (not timed).
    Returns (seconds, gradient)."""
    D = theta32.size
    s = np.float32(sigma)
    vecs = np.empty((len(indices), D), np.float32)
    for i, idx in enumerate(indices):
        np.multiply(s, table[idx: idx + D], out=vecs[i])
    theta = theta32.copy()
    m = np.zeros(D, np.float64)
    v = np.zeros(D, np.float64)
    t0 = time.perf_counter()
    cr = _centered_ranks(np.asarray(fitness, np.float64))
    w = cr[:, 0] - cr[:, 1]
    total = 0.
    for k in range(0, len(indices), 500):
        total += np.dot(np.asarray(w[k:k + 500], dtype=np.float32), vecs[k:k + 500])
    g = total / cr.size
    globalg = -g + l2coeff * theta
    a = stepsize * np.sqrt(1 - 0.999) / (1 - 0.9)
    m = 0.9 * m + (1 - 0.9) * globalg
    v = 0.999 * v + (1 - 0.999) * (globalg * globalg)
    step = -a * m / (np.sqrt(v) + 1e-08)
    _ = np.linalg.norm(step) / np.linalg.norm(theta)
    theta = theta + step
    secs = time.perf_counter() - t0
    return secs, g
