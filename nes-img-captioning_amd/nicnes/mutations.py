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
weighted noise sum and nicnes_noise_vectors then read). The SM-G-SUM vector s is computed once per
task, as the reference's workers do (nic_nes_worker.py:137-140), by the engine itself
(Engine.sum_sensitivity -> nicnes_sum_sensitivity: the Jacobian of 95 grouped log-prob outputs after 5
greedy steps, CaptionModel.forward_for_sensitivity, src/captioning/nets.py:22-70, its 95 backward
passes batched on the GPU); oracle/sensitivity_ref.py keeps the torch-autograd restatement in the
reference's op order that pins it (bit-exact vs the reference's calc_sensitivity).

One sensitivity per task: the reference caches it per (task, parent 0) in a file shared by the
workers (safe_mutations.py:34-52), so every member uses the first worker's batch; with
single_batch: false the engine uses the iteration's first batch for it (batch 0).
"""
import numpy as np
import torch

SAFE_DIVIDE = ('SM-G-SUM', 'SM-VECTOR')
MODES = ('', 'SM-G-SUM', 'SM-G-ABS', 'SM-VECTOR', 'SM-PROPORTIONAL')


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


def proportional_mean(theta32):
    """mean|theta| in fp32 as torch computes it on the host (nets.py:110), the value exact zeros take."""
    if isinstance(theta32, torch.Tensor):
        return theta32.detach().to('cpu', torch.float32).abs().mean()
    return torch.as_tensor(np.asarray(theta32, np.float32)).abs().mean()


def proportional_vector(theta32):
    """nets.py:108-112: |theta| with exact zeros replaced by mean|theta| (the mean in fp32, as torch)."""
    p = torch.as_tensor(np.asarray(theta32, np.float32)).clone()
    mean = p.abs().mean()
    p[p == 0.0] = mean
    return p.abs()


class Mutator:
    """Sets the engine's noise transform for each task (nets.py:83-119 semantics).

    prepare(key, theta32, fc_unique) is called with the task's fp32 theta (loaded in the engine) and its
    (first) batch's unique fc rows (the batch the engine holds) before the task's members are evaluated
    or summed; the vector is recomputed only when `key` changes. Workers and the master compute the
    vector from the same inputs with the same engine code, so the master's weighted noise sum uses the
    workers' noise."""

    def __init__(self, spec, engine):
        mo = spec.model_options
        self.mode = mo.safe_mutations or ''
        self.e = engine
        self.underflow = float(mo.safe_mutation_underflow or 0.0)
        self.orig_bs = spec.batch_size                   # Experiment.orig_batch_size (experiment.py:29,110)
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
        """theta32: the fp32 theta, or a callable returning it (read only by SM-PROPORTIONAL: SM-G-SUM takes theta
        from the engine itself, so the callers pass `lambda: engine.theta()[1]` and no copy is made for it)."""
        if not self.active or key == self._key:
            return self.vector
        if self.mode == 'SM-PROPORTIONAL':
            def theta_now():
                return theta32() if callable(theta32) else theta32
            if hasattr(self.e, 'set_mutation_proportional'):
                # the engine forms |theta'| from its own theta on the device; the host computes only the mean,
                # and only when theta has exact zeros for it to replace (4.1 ms a task with the vector's host
                # round trip at D = 2.87 M; 1.9 ms with the mean; tens of us without). theta is read only then.
                mean = float(proportional_mean(theta_now())) if self.e.theta_zeros() else 0.0
                self.e.set_mutation_proportional(mean)
                self.vector = None
            else:
                th = theta_now()
                th = th.detach().cpu().numpy() if isinstance(th, torch.Tensor) else np.asarray(th)
                self.vector = proportional_vector(th.astype(np.float32, copy=False))
                self.e.set_mutation('scale', self.vector)
        else:
            if not self.underflow > 0:
                raise ValueError('SM-G-SUM needs safe_mutation_underflow > 0 (the reference divides by it)')
            # forward_for_sensitivity's rows: the batch's unique images, the first orig_batch_size of them
            rows = int(np.asarray(fc_unique).shape[0])
            if rows > self.orig_bs > 0:
                rows = self.orig_bs
            self.vector = self.e.sum_sensitivity(rows, self.underflow)
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
