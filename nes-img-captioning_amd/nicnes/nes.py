"""Reference-facing NIC-NES objects backed by the engine (the drop-in boundary, host side).

Mirrors the interfaces of rubencart/NES-img-captioning that the fc_caption NES hot path goes
through, with the same names, argument meaning and error behaviour:

  NESTask / NESResult        /root/reference/src/algorithm/nic_nes/nic_nes_master.py:27-31
  EnginePolicy               Policy (/root/reference/src/algorithm/policies.py:44-172) and
                             CaptPolicy.rollout (/root/reference/src/captioning/policies.py:86-128)
  EngineWorker.fitness       NESWorker.fitness (/root/reference/src/algorithm/nic_nes/nic_nes_worker.py:115-161)
  gradient_estimate & co     NESMaster.gradient_estimate / compute_centered_ranks / compute_ranks
                             (nic_nes_master.py:170-205)
  Adam / SGD                 Optimizer.update / save_to_file / load_from_file (optimizers.py:8-107)

The one contract change: a result carries the member's noise-table offset (`noise_idx`) instead
of the 11 MB `evolve_noise` vector; the master rebuilds delta from the shared table.
"""
import os
from collections import OrderedDict, namedtuple

import numpy as np
import torch

nes_task_fields = ['current', 'batch_data', 'noise_stdev', 'log_dir', 'ref_batch', 'batch_size', 'iteration']
NESTask = namedtuple('NESTask', field_names=nes_task_fields, defaults=(None,) * len(nes_task_fields))

result_fields = ['worker_id', 'eval_score', 'evolve_noise', 'fitness', 'mem_usage', 'noise_idx', 'member']
NESResult = namedtuple('NESResult', field_names=result_fields, defaults=(None,) * len(result_fields))

PARAM_NAMES = ['img_embed.weight', 'img_embed.bias', 'embed.weight', 'logit.weight', 'logit.bias',
               'core.i2h.weight', 'core.i2h.bias', 'core.h2h.weight', 'core.h2h.bias']


# ---------------------------------------------------------------- theta <-> state_dict ----------
def param_shapes(engine):
    c = engine.cfg
    V1, E, R, F = c.vocab_size + 1, c.input_encoding_size, c.rnn_size, c.fc_feat_size
    return OrderedDict([('img_embed.weight', (E, F)), ('img_embed.bias', (E,)), ('embed.weight', (V1, E)),
                        ('logit.weight', (V1, R)), ('logit.bias', (V1,)), ('core.i2h.weight', (5 * R, E)),
                        ('core.i2h.bias', (5 * R,)), ('core.h2h.weight', (5 * R, R)), ('core.h2h.bias', (5 * R,))])


def vector_from_state_dict(sd, shapes):
    """parameters_to_vector in FCModel registration order (nets.py:150-153, LSTMCore :81-82)."""
    parts = []
    for name, shp in shapes.items():
        if name not in sd:
            raise KeyError('state_dict lacks %r (vbn / layer-norm models are not supported)' % name)
        t = sd[name]
        t = t.detach().cpu() if isinstance(t, torch.Tensor) else torch.from_numpy(np.asarray(t))
        if tuple(t.shape) != tuple(shp):
            raise ValueError('%s has shape %s, expected %s' % (name, tuple(t.shape), shp))
        parts.append(t.reshape(-1))
    return torch.cat(parts)


def state_dict_from_vector(vec, shapes):
    sd, o = OrderedDict(), 0
    vec = vec.detach().cpu() if isinstance(vec, torch.Tensor) else torch.from_numpy(np.asarray(vec))
    for name, shp in shapes.items():
        n = int(np.prod(shp))
        sd[name] = vec[o:o + n].reshape(shp).clone()
        o += n
    return sd


def unique_batch(data, seq_per_img=5):
    """Reference batch dict (dataloader.get_batch, dataloader.py:135-203: fc_feats [B*5, F], gts
    list of [n_i, 16]) -> (unique fc [B, F] fp32, gts). Greedy decoding of duplicated rows is
    deterministic, so one row per image gives the same tokens and, in fixed-df CIDEr-D, the same
    mean fitness."""
    fc = np.asarray(data['fc_feats'], np.float32)
    gts = data['gts']
    if fc.shape[0] == len(gts) * seq_per_img and seq_per_img > 1:
        fc = fc[::seq_per_img]
    if fc.shape[0] != len(gts):
        raise ValueError('fc_feats rows (%d) do not match the %d images of gts' % (fc.shape[0], len(gts)))
    return np.ascontiguousarray(fc), gts


SAMPLED_FITNESS_CODES = (5, 6, 7)     # 'sample', 'self_critical', 'sc_loss' (nicnes.h NICNES_FITNESS_*)


def engine_batch(data, engine, seq_per_img=5):
    """The images the engine holds for a reference batch dict (unique_batch). The sampled modes decode every
    copy of an image, so the engine is told how many rows each image has (Engine.set_rows_per_image, the
    batch's seq_per_img); the copies are not uploaded."""
    fc, gts = unique_batch(data, seq_per_img)
    if getattr(engine, 'fitness_mode', 0) in SAMPLED_FITNESS_CODES and hasattr(engine, 'set_rows_per_image'):
        engine.set_rows_per_image(max(1, np.asarray(data['fc_feats']).shape[0] // len(gts)))
    return fc, gts


def member_batches(batch_data, member_begin, count):
    """Per-member batch indices when batch_data is a list of G batches (member i uses batch i mod G),
    None for one shared batch."""
    if isinstance(batch_data, (list, tuple)) and len(batch_data) > 1:
        return [(member_begin + k) % len(batch_data) for k in range(count)]
    return None


# ---------------------------------------------------------------- policy (Policy API) ------------
class ParameterFileError(OSError):
    """The parameter file could not be read as a state_dict: the master deletes and rewrites it between
    iterations (nic_nes_worker.py:71-84), so a late reader can find it half written. Transient; nothing
    else a worker raises is."""


class EnginePolicy:
    """Policy / CaptPolicy for the engine: theta lives on the GPU (fp64 master + fp32 copy)."""

    def __init__(self, engine, spec=None):
        self.e = engine
        self.spec = spec
        self.shapes = param_shapes(engine)
        self._batch_key = None
        # the eval rollouts' draw stream (sampled modes): a per-process random start, so two workers sharing
        # --noise_seed, or a restarted worker, do not replay each other's draws -- each reference worker process
        # draws from its own unseeded RandomState (nic_nes_worker.py:22). The engine hashes the low 32 bits.
        self._eval_salt = int.from_bytes(os.urandom(4), 'little')
        self._eval_calls = 0
        if spec is not None:
            engine.set_fitness_mode(spec.fitness)      # CaptPolicy's Fitness (policies.py:22-61)

    # Policy.set_model (policies.py:125-147): PolicyNet-like object, state_dict, or .pth path
    def set_model(self, model):
        if isinstance(model, str):
            import pickle
            try:
                model = torch.load(model, map_location='cpu', weights_only=True)
            except FileNotFoundError:
                raise
            except (EOFError, OSError, RuntimeError, pickle.UnpicklingError) as e:
                # a truncated zip archive or pickle stream (torch.load's errors for a half-written file: a seek past
                # the end, a missing central directory, a cut pickle)
                raise ParameterFileError('parameter file %s unreadable: %s' % (model, e)) from e
        elif hasattr(model, 'state_dict') and not isinstance(model, dict):
            model = model.state_dict()
        if not isinstance(model, dict):
            raise AssertionError('{}'.format(type(model)))
        vec = vector_from_state_dict(model, self.shapes)
        self.e.set_theta(vec.numpy() if vec.dtype == torch.float32 else vec.double().numpy())

    def parameter_vector(self):
        """fp32 evaluation copy (what workers evaluate, nic_nes_worker.py:130-132)."""
        return self.e.theta()[1]

    def set_from_parameter_vector(self, vector):
        assert isinstance(vector, (np.ndarray, torch.Tensor))
        self.e.set_theta(vector)

    def state_dict(self):
        return state_dict_from_vector(self.e.theta()[1], self.shapes)

    def serialize(self, path):
        torch.save(self.state_dict(), path)
        return path

    def nb_learnable_params(self):
        return self.e.D

    def evolve_model(self, sigma, iteration=0, member=0):
        """The member's perturbation is fp32(sigma * table[idx : idx + D]); returns idx (the noise
        index replaces the returned noise vector of PolicyNet.evolve, nets.py:83-119)."""
        return int(self.e.noise_indices(iteration, member, 1).cpu()[0])

    def _ensure_batch(self, data, seq_per_img=5):
        """Load the batch (a reference batch dict) or the batches (a list of them, single_batch: false)
        unless this very object is already loaded. The object itself is kept: an id() of a freed batch
        can be reused by the next one."""
        if data is not self._batch_key:
            if isinstance(data, (list, tuple)):
                ub = [engine_batch(d, self.e, seq_per_img) for d in data]
                if len(ub) == 1:
                    self.e.set_batch(*ub[0])
                else:
                    self.e.set_batches(ub)
                rows = ub[0][0].shape[0]
            else:
                fc, gts = engine_batch(data, self.e, seq_per_img)
                self.e.set_batch(fc, gts)
                rows = fc.shape[0]
            self._batch_key = data
            self._batch_rows = rows
        return self._batch_rows

    def eval_iteration(self):
        """The draw-stream index of the newest eval rollout: this process's salt + its call count (mod 2^32)."""
        return (self._eval_salt + self._eval_calls) & 0xffffffff

    def rollout(self, placeholder, data, config):
        """CaptPolicy.rollout (policies.py:86-128) of the current theta: float(100 * mean CIDEr-D) for
        'greedy' and 'sample', 100 * the mean self-critical difference for 'self_critical', the criterion
        value for the greedy_* modes and 'sc_loss'."""
        self._ensure_batch(data)
        # theta itself, decoded once (nicnes_evaluate_theta: the two antithetic signs split the images);
        # with several batches held, member 0's batch (member_batches' rule)
        # the sampled modes draw afresh per eval rollout, as the reference's worker RNG does
        self._eval_calls += 1
        fit = self.e.evaluate_theta(0, iteration=self.eval_iteration())
        return float(fit[0].item())


# ---------------------------------------------------------------- worker --------------------------
class EngineWorker:
    """NESWorker.fitness over populations: one call evaluates members [member_begin, +count)."""

    def __init__(self, engine, spec=None, worker_id=None):
        self.e = engine
        self.spec = spec
        self.worker_id = worker_id if worker_id is not None else os.getpid()
        self.policy = EnginePolicy(engine, spec)
        self.mutator = None
        if spec is not None and spec.mutation:
            from .mutations import Mutator
            self.mutator = Mutator(spec, engine)

    def _prepare(self, task_id, task_data):
        # theta and batch are loaded once per task (the reference reloads them per member)
        cur = task_data.current
        prev = getattr(self, '_cur', None)
        # a path is compared by value within a task; any other model object by identity (kept alive)
        same = prev is not None and prev[0] == task_id and (prev[1] == cur if isinstance(cur, str) else prev[1] is cur)
        if cur is not None and not same:
            self.policy.set_model(cur)
            self._cur = (task_id, cur)
            self._cur_version = getattr(self, '_cur_version', 0) + 1
        if task_data.batch_data is not None:
            self.policy._ensure_batch(task_data.batch_data)
        if self.mutator is not None and self.mutator.active:
            # calc_sensitivity of the task's theta on its batch before evolve (nic_nes_worker.py:137-142)
            from .mutations import batch_fc
            self.mutator.prepare((task_id, getattr(self, '_cur_version', 0)), lambda: self.e.theta()[1],
                                 batch_fc(task_data.batch_data))

    def fitness_batch(self, task_id, task_data, member_begin, count, batches=None):
        """-> list of NESResult(fitness=[f+, f-] fp64, noise_idx, member). batches (single_batch: false on the
        reference wire): one batch dict per member, member k scored on batches[k] -- each drawn from the worker's
        own loader, as each reference fitness call draws one (nic_nes_worker.py:121-128)."""
        mb = None
        if batches is not None:
            if len(batches) != count:
                raise ValueError('one batch per member: %d batches for %d members' % (len(batches), count))
            task_data = task_data._replace(batch_data=list(batches))
            mb = list(range(count)) if count > 1 else None
        self._prepare(task_id, task_data)
        it = int(task_data.iteration if task_data.iteration is not None else task_id)
        if mb is None:
            mb = member_batches(task_data.batch_data, member_begin, count)
        fit = self.e.evaluate(it, member_begin, count, float(task_data.noise_stdev), member_batch=mb).cpu().numpy()
        idx = self.e.noise_indices(it, member_begin, count).cpu().numpy()
        return [NESResult(worker_id=self.worker_id, fitness=fit[k].copy(), noise_idx=int(idx[k]),
                          member=member_begin + k) for k in range(count)]

    def fitness(self, task_id, policy, task_data, member=0):
        """Same call shape as NESWorker.fitness(task_id, policy, task_data) for one member."""
        return self.fitness_batch(task_id, task_data, member, 1)[0]


# ---------------------------------------------------------------- master ops ----------------------
def compute_ranks(engine, x):
    """nic_nes_master.py:196-205 (stable tie-break); x 1-d, even length -> int ranks."""
    x = np.asarray(x, np.float64).ravel()
    cr = compute_centered_ranks(engine, x.reshape(-1, 2))
    return np.rint((cr.ravel() + 0.5) * (x.size - 1)).astype(int)


def compute_centered_ranks(engine, x):
    """nic_nes_master.py:184-194 on the GPU rank kernel; x (F, 2) -> (F, 2) fp64."""
    x = np.ascontiguousarray(np.asarray(x, np.float64).reshape(-1, 2))
    cr, _ = engine.rank_weights(torch.from_numpy(x).to(engine.device))
    return cr.cpu().numpy()


def gradient_estimate(engine, fitnesses, noise_indices, sigma, iteration, member_begin=0):
    """NESMaster.gradient_estimate (nic_nes_master.py:170-182) with deltas re-read from the table.
    `noise_indices` must be the engine's own indices for (iteration, member_begin + i) -- checked.
    Returns g = sum_i w_i delta_i / (2F) as an fp32 device tensor."""
    fit = torch.from_numpy(np.ascontiguousarray(np.asarray(fitnesses, np.float64))).to(engine.device)
    F = fit.shape[0]
    want = engine.noise_indices(iteration, member_begin, F).cpu().numpy()
    if noise_indices is not None and not np.array_equal(np.asarray(noise_indices, np.int64), want):
        raise ValueError('noise indices do not follow the engine rule for this iteration/member range')
    _, w = engine.rank_weights(fit)
    gsum = engine.grad_partial(iteration, member_begin, F, w, sigma)
    return gsum / torch.tensor(2 * F, dtype=torch.float32, device=engine.device)


# ---------------------------------------------------------------- optimizers -----------------------
class _EngineOptimizer:
    kind = None

    def __init__(self, engine, theta=None):
        self.e = engine
        if theta is not None:
            self.set_theta(theta)

    @property
    def dim(self):
        return self.e.D

    @property
    def t(self):
        return self.e.adam_state()[2]

    @property
    def theta(self):
        return self.e.theta()[0].cpu().numpy()

    def set_theta(self, theta):
        self.e.set_theta(theta)

    def update(self, globalg):
        """Optimizer.update(globalg) -> (ratio, theta fp64)."""
        ratio = self.e.optimizer_update(globalg, self.kind, **self._args())
        return ratio, self.theta

    def update_from_noise_sum(self, gsum, P, l2coeff):
        """Fused NES form: globalg = -gsum/(2P) + l2coeff*theta, computed on the GPU."""
        raise NotImplementedError


class Adam(_EngineOptimizer):
    kind = 'adam'

    def __init__(self, engine, theta=None, stepsize=1e-3, beta1=0.9, beta2=0.999, epsilon=1e-08):
        self.stepsize, self.beta1, self.beta2, self.epsilon = stepsize, beta1, beta2, epsilon
        super().__init__(engine, theta)

    def _args(self):
        return dict(stepsize=self.stepsize, beta1=self.beta1, beta2=self.beta2, epsilon=self.epsilon)

    def update_from_noise_sum(self, gsum, P, l2coeff):
        return self.e.adam_step(gsum, P, l2coeff, self.stepsize, self.beta1, self.beta2, self.epsilon)

    def save_to_file(self, path):
        """optimizer.tar with the reference keys and types (optimizers.py:85-95): m, v as fp64 numpy
        arrays, so the reference's load_from_file gets the numpy state it expects."""
        m, v, t = self.e.adam_state()
        torch.save({'dim': self.dim, 't': t, 'stepsize': self.stepsize, 'beta1': self.beta1, 'beta2': self.beta2,
                    'epsilon': self.epsilon, 'm': m.cpu().numpy(), 'v': v.cpu().numpy()}, path)

    def load_from_file(self, path):
        state = _load_state(path)
        self.stepsize, self.beta1, self.beta2, self.epsilon = (state['stepsize'], state['beta1'], state['beta2'],
                                                               state['epsilon'])
        self.e.set_adam_state(np.asarray(state['m'], np.float64), np.asarray(state['v'], np.float64), state['t'])


class SGD(_EngineOptimizer):
    kind = 'sgd'

    def __init__(self, engine, theta=None, stepsize=1e-3, momentum=0.9):
        self.stepsize, self.momentum = stepsize, momentum
        super().__init__(engine, theta)

    def _args(self):
        return dict(stepsize=self.stepsize, beta1=self.momentum, beta2=0.0, epsilon=0.0)

    def update_from_noise_sum(self, gsum, P, l2coeff):
        return self.e.sgd_step(gsum, P, l2coeff, self.stepsize, self.momentum)

    def save_to_file(self, path):
        _, v, t = self.e.adam_state()
        torch.save({'dim': self.dim, 't': t, 'momentum': self.momentum, 'stepsize': self.stepsize,
                    'v': v.cpu().numpy()}, path)

    def load_from_file(self, path):
        state = _load_state(path)
        self.stepsize, self.momentum = state['stepsize'], state['momentum']
        v = np.asarray(state['v'], np.float64)
        self.e.set_adam_state(np.zeros_like(v), v, state['t'])


def _load_state(path):
    """torch.load with weights_only=True; numpy arrays (the reference saves m, v as ndarrays) are
    admitted through the safe-globals allowlist, nothing is unpickled beyond that."""
    import numpy.core.multiarray as ma
    allow = [ma._reconstruct, np.ndarray, np.dtype, type(np.dtype(np.float64))]
    with torch.serialization.safe_globals(allow):
        state = torch.load(path, map_location='cpu', weights_only=True)
    return {k: (v.numpy() if isinstance(v, torch.Tensor) else v) for k, v in state.items()}


def make_optimizer(engine, spec, theta=None):
    """NESExperiment's {'sgd': SGD, 'adam': Adam}[type](theta, **args) (nic_nes/experiment.py:20-21)."""
    cls = {'adam': Adam, 'sgd': SGD}[spec.optimizer_type]
    return cls(engine, theta, **spec.optimizer_args)
