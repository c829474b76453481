"""Safe and proportional mutations (model_options.safe_mutations) for the engine.

PolicyNet.evolve (src/algorithm/nets.py:83-119) transforms the member's noise before theta +/- noise:

  SM-G-SUM         noise / s, s = the output-gradient sensitivity of the current theta on the task
                   batch (Sensitivity.calc_sensitivity + _calc_sum_sensitivity, safe_mutations.py:34-117)
  SM-VECTOR        noise / s, s = a sensitivity file (Sensitivity.set_sensitivity, safe_mutations.py:27-31)
  SM-PROPORTIONAL  noise * |theta'|, theta' = theta with exact zeros replaced by mean|theta| (nets.py:108-112)
  SM-G-ABS         not offered: the reference's _calc_abs_sensitivity reads self.nb_params on the
                   Sensitivity object (safe_mutations.py:125), which has none, so it raises
                   AttributeError before producing a vector.

The engine applies the transform on the GPU (nicnes_set_mutation: one prepass materialises
fp32(fp32(sigma * z) / s) or fp32(fp32(sigma * z) * |theta'|) per member, which the decode, the
weighted noise sum and nicnes_noise_vectors then read). This module computes the per-parameter
vector s on the host once per task, as the reference's workers do (nic_nes_worker.py:137-140):
the sensitivity is a Jacobian of 95 grouped log-prob outputs after 5 greedy steps
(CaptionModel.forward_for_sensitivity, src/captioning/nets.py:22-70) -- 95 backward passes of a
5-step decode on at most orig_batch_size images, taken with torch autograd on the CPU in the
reference's own op order, so the vector is the reference's vector.

One sensitivity per task: the reference caches it per (task, parent 0) in a file shared by the
workers (safe_mutations.py:34-52), so every member uses the first worker's batch; with
single_batch: false the engine uses the iteration's first batch for it (batch 0).
"""
import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

SAFE_DIVIDE = ('SM-G-SUM', 'SM-VECTOR')
MODES = ('', 'SM-G-SUM', 'SM-G-ABS', 'SM-VECTOR', 'SM-PROPORTIONAL')


class _Core(nn.Module):
    """LSTMCore without vbn / layer norm (src/captioning/nets.py:75-134)."""

    def __init__(self, E, R):
        super().__init__()
        self.R = R
        self.i2h = nn.Linear(E, 5 * R)
        self.h2h = nn.Linear(R, 5 * R)

    def forward(self, xt, h, c):
        s = self.i2h(xt) + self.h2h(h)
        g = torch.sigmoid(s.narrow(1, 0, 3 * self.R))
        ig, fg, og = g.narrow(1, 0, self.R), g.narrow(1, self.R, self.R), g.narrow(1, 2 * self.R, self.R)
        tr = torch.max(s.narrow(1, 3 * self.R, self.R), s.narrow(1, 4 * self.R, self.R))
        c = fg * c + ig * tr
        return og * torch.tanh(c), c


class SensitivityNet(nn.Module):
    """The fc_caption parameters in FCModel registration order (nets.py:150-153), differentiable,
    for the sensitivity Jacobian only (the engine's decode runs on the GPU)."""

    def __init__(self, V1, E, R, F_):
        super().__init__()
        self.R = R
        self.img_embed = nn.Linear(F_, E)
        self.embed = nn.Embedding(V1, E)
        self.logit = nn.Linear(R, V1)
        self.core = _Core(E, R)

    def load_vector(self, theta32):
        nn.utils.vector_to_parameters(torch.as_tensor(np.asarray(theta32, np.float32)), self.parameters())

    def forward_for_sensitivity(self, fc_unique, orig_bs=0, split=100, length=5):
        """captioning/nets.py:22-70 on unique image rows: log-probs after `length` greedy steps, the
        vocabulary zero-padded to a multiple of `split` and each group reduced to its 2-norm."""
        fc = torch.as_tensor(np.ascontiguousarray(fc_unique, np.float32))
        if fc.size(0) > orig_bs > 0:
            fc = fc[:orig_bs]
        B = fc.size(0)
        h = fc.new_zeros(B, self.R)
        c = fc.new_zeros(B, self.R)
        h, c = self.core(self.img_embed(fc), h, c)
        it = torch.zeros(B, dtype=torch.long)
        for _ in range(length):
            h, c = self.core(self.embed(it), h, c)
            logprobs = F.log_softmax(self.logit(h), dim=1)
            _, it = torch.max(logprobs.data, 1)
            it = it.view(-1).long()
        pad = split - (logprobs.size(1) % split)
        ext = torch.cat((logprobs, torch.zeros((B, pad))), 1)
        return ((torch.stack(ext.split(split, dim=1)) ** 2).sum(2) ** (1 / 2)).permute(1, 0)

    def extract_grad(self):
        return torch.cat([p.grad.data.flatten() for p in self.parameters()])


def sum_sensitivity(dims, theta32, fc_unique, orig_bs):
    """Sensitivity._calc_sum_sensitivity (safe_mutations.py:86-110): per parameter, the 2-norm over
    the grouped outputs of d(output summed over the batch)/d(theta), divided by the batch size.
    dims = (V1, E, R, F). Returns fp32 [D] (before the underflow clamp)."""
    net = SensitivityNet(*dims)
    net.load_vector(theta32)
    with torch.enable_grad():
        for p in net.parameters():
            p.requires_grad_(True)
        out = net.forward_for_sensitivity(fc_unique, orig_bs)
        n_out, B = out.size(1), out.size(0)
        D = sum(p.numel() for p in net.parameters())
        jac = torch.zeros(n_out, D)
        go = torch.zeros(*out.size())
        for k in range(n_out):
            net.zero_grad()
            go.zero_()
            go[:, k] = 1.0
            out.backward(gradient=go, retain_graph=True)
            jac[k] = net.extract_grad()
    s = torch.sqrt((jac ** 2).sum(0))
    s /= B
    return s.detach()


def clamp_calc(s, underflow):
    """Sensitivity.calc_sensitivity (safe_mutations.py:63-65): s < underflow -> underflow, / underflow."""
    if not underflow > 0:
        raise ValueError('SM-G-SUM needs safe_mutation_underflow > 0 (the reference divides by it)')
    s = s.clone()
    s[s < underflow] = underflow
    s /= underflow
    return s


def clamp_file(s, underflow):
    """Sensitivity.set_sensitivity (safe_mutations.py:27-31): s < underflow -> underflow, / min."""
    s = s.clone().float()
    s[s < underflow] = underflow
    s /= s.min()
    return s


def load_vector_file(path, underflow):
    """SM-VECTOR's file: a tensor saved with torch.save (read with weights_only=True), or .npy."""
    if str(path).endswith('.npy'):
        s = torch.from_numpy(np.load(path).astype(np.float32))
    else:
        s = torch.load(path, map_location='cpu', weights_only=True)
    return clamp_file(s.reshape(-1), underflow)


def proportional_vector(theta32):
    """nets.py:108-112: |theta| with exact zeros replaced by mean|theta| (the mean in fp32, as torch)."""
    p = torch.as_tensor(np.asarray(theta32, np.float32)).clone()
    mean = p.abs().mean()
    p[p == 0.0] = mean
    return p.abs()


class Mutator:
    """Sets the engine's noise transform for each task (nets.py:83-119 semantics).

    prepare(key, theta32, fc_unique) is called with the task's fp32 theta and its (first) batch's
    unique fc rows before the task's members are evaluated or summed; the vector is recomputed only
    when `key` changes. Workers and the master compute the same vector from the same inputs (CPU
    torch, deterministic), so the master's weighted noise sum uses the workers' noise."""

    def __init__(self, spec, engine):
        mo = spec.model_options
        self.mode = mo.safe_mutations or ''
        self.e = engine
        self.underflow = float(mo.safe_mutation_underflow or 0.0)
        self.orig_bs = spec.batch_size                   # Experiment.orig_batch_size (experiment.py:29,110)
        c = engine.cfg
        self.dims = (c.vocab_size + 1, c.input_encoding_size, c.rnn_size, c.fc_feat_size)
        self._key = None
        self.vector = None
        if self.mode == 'SM-VECTOR':
            if not mo.safe_mutation_vector:
                raise ValueError('SM-VECTOR needs model_options.safe_mutation_vector')
            self.vector = load_vector_file(mo.safe_mutation_vector, self.underflow)
            engine.set_mutation('divide', self.vector)

    @property
    def active(self):
        return self.mode in ('SM-G-SUM', 'SM-PROPORTIONAL')

    def prepare(self, key, theta32, fc_unique):
        if not self.active or key == self._key:
            return self.vector
        th = theta32.detach().cpu().numpy() if isinstance(theta32, torch.Tensor) else np.asarray(theta32)
        th = th.astype(np.float32, copy=False)
        if self.mode == 'SM-PROPORTIONAL':
            self.vector = proportional_vector(th)
            self.e.set_mutation('scale', self.vector)
        else:
            s = sum_sensitivity(self.dims, th, fc_unique, self.orig_bs)
            self.vector = clamp_calc(s, self.underflow)
            self.e.set_mutation('divide', self.vector)
        self._key = key
        return self.vector


def batch_fc(batch):
    """Unique fc rows of a task batch: a reference batch dict, (fc, gts), or a list of either (the first)."""
    from .nes import unique_batch
    if isinstance(batch, list):
        batch = batch[0]
    if isinstance(batch, dict):
        return unique_batch(batch)[0]
    return np.asarray(batch[0], np.float32)
