"""TEST INFRASTRUCTURE (oracle): the SM-G-SUM sensitivity restated with torch autograd on the CPU.

Follows Sensitivity._calc_sum_sensitivity (/root/reference/src/algorithm/safe_mutations.py:93-117) on
CaptionModel.forward_for_sensitivity (/root/reference/src/captioning/nets.py:22-70) and LSTMCore
(nets.py:75-134) in the reference's op order; tests/golden/mutations.npz pins it bit for bit against the
reference's own calc_sensitivity. The engine computes the same vector on the GPU
(nicnes_sum_sensitivity); only tests/ and tests/cpu_engine.py's OracleEngine use this module.
"""
import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F


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
    """Sensitivity._calc_sum_sensitivity (safe_mutations.py:93-117): per parameter, the 2-norm over
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
