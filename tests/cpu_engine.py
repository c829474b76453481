"""Test helper: an Engine look-alike on CPU tensors built from the oracle (test infrastructure only),
so the sharded PopulationRunner logic (nicnes/population.py) can run over gloo without a GPU."""
import numpy as np
import torch

from oracle import cider_ref as CR
from oracle import oracle as O


class _Cfg:
    def __init__(self, dims):
        self.vocab_size, self.input_encoding_size, self.rnn_size, self.fc_feat_size = dims.vocab_size, dims.E, \
            dims.R, dims.F
        self.seq_length = 16


class OracleEngine:
    def __init__(self, dims, theta32, fc, gts, df, ref_len_raw, table, noise_seed=0):
        self.device = torch.device('cpu')
        self.dims, self.D = dims, dims.D
        self.cfg = _Cfg(dims)
        self.fc, self.gts, self.table, self.seed = fc, gts, table, noise_seed
        self.scorer = CR.CiderDOracle(df, ref_len_raw)
        self.adam = None
        self.theta32 = theta32.copy()
        self.theta_src = theta32.copy()
        self.fitness_mode = 0
        self.mutation = None

    def set_mutation(self, mode='plain', vec=None):
        v = vec.numpy() if isinstance(vec, torch.Tensor) else vec
        self.mutation = None if mode == 'plain' else (mode, np.asarray(v, np.float32).copy())

    def sum_sensitivity(self, rows, underflow=0.0):
        """nicnes_sum_sensitivity on the CPU: the torch-autograd oracle (oracle/sensitivity_ref.py) on the
        first `rows` images of the batch held."""
        from nicnes.mutations import clamp_calc
        from oracle import sensitivity_ref as SR
        d = self.dims
        fc = self.batches[0][0] if getattr(self, 'batches', None) else np.asarray(self.fc)   # batch 0
        s = SR.sum_sensitivity((d.vocab_size + 1, d.E, d.R, d.F), self.theta32, fc[:rows], rows)
        return clamp_calc(s, underflow) if underflow > 0 else s

    def set_rows_per_image(self, n=1):
        self.rpi = int(n)

    def set_fitness_mode(self, fitness):
        self.fitness_mode = CR.CRITERIA[fitness] if isinstance(fitness, str) else int(fitness)

    # ---- Engine surface used by nicnes.nes / nicnes.master
    def set_theta(self, theta, fp32_origin=None):
        th = theta.numpy() if isinstance(theta, torch.Tensor) else np.asarray(theta)
        self.theta_src = th.copy()
        self.theta32 = th.astype(np.float32)
        self.adam = None

    def theta(self):
        src = self.adam.theta if self.adam is not None else self.theta_src
        return torch.from_numpy(np.asarray(src, np.float64).copy()), torch.from_numpy(self.theta32.copy())

    def set_batch(self, fc, gts):
        self.fc, self.gts = np.asarray(fc, np.float32), gts
        self.batches = None

    def set_batches(self, batches):
        self.batches = [(np.asarray(f, np.float32), g) for f, g in batches]

    def noise_indices(self, iteration, member_begin, count):
        return torch.tensor([self._idx(iteration, member_begin + k) for k in range(count)], dtype=torch.int64)

    def noise_vectors(self, iteration, member_begin, count, sigma, out=None):
        v = np.stack([O.member_delta(self.table, self._idx(iteration, member_begin + k), sigma, self.D, self.mutation)
                      for k in range(count)])
        return torch.from_numpy(v)

    def adam_state(self):
        if self.adam is None:
            z = torch.zeros(self.D, dtype=torch.float64)
            return z, z.clone(), 0
        m = getattr(self.adam, 'm', np.zeros(self.D))
        return torch.from_numpy(np.asarray(m, np.float64)), torch.from_numpy(self.adam.v.copy()), self.adam.t

    def sgd_step(self, gsum, P, l2coeff, stepsize, momentum=0.9):
        if self.adam is None:
            self.adam = O.SGDOracle(self.theta_src.copy(), stepsize, momentum)
        self.adam.stepsize, self.adam.momentum = stepsize, momentum      # a schedule may change them
        g = gsum.numpy().astype(np.float32) / np.float32(2 * P)
        ratio, theta = O.master_update(self.adam, g, l2coeff)
        self.theta32 = np.asarray(theta).astype(np.float32)
        return float(ratio)

    def _idx(self, iteration, m):
        return O.noise_index(self.seed, iteration, m, self.table.size, self.D)

    def evaluate(self, iteration, member_begin, count, sigma, fitness_out=None, member_batch=None):
        out = fitness_out if fitness_out is not None else torch.empty((count, 2), dtype=torch.float64)
        for k in range(count):
            idx = self._idx(iteration, member_begin + k)
            fc, gts = (self.fc, self.gts) if member_batch is None else self.batches[member_batch[k]]
            for s, sign in enumerate((+1, -1)):
                seq, lp, _ = O.decode(self.dims, O.perturb(self.theta32, self.table, idx, sigma, sign, self.mutation), fc)
                f, scores = CR.rollout_fitness(self.scorer, seq, gts)
                out[k, s] = CR.criterion_fitness(self.fitness_mode, lp, seq, scores) if self.fitness_mode else f
        return out

    def evaluate_theta(self, batch=0, iteration=0):
        fc, gts = (self.fc, self.gts) if not getattr(self, 'batches', None) else self.batches[batch]
        seq, lp, _ = O.decode(self.dims, self.theta32, fc)
        f, scores = CR.rollout_fitness(self.scorer, seq, gts)
        return torch.tensor([CR.criterion_fitness(self.fitness_mode, lp, seq, scores) if self.fitness_mode else f],
                            dtype=torch.float64)

    def rank_weights(self, fitness_all):
        w, cr = O.weights_from_fitness(fitness_all.numpy())
        return torch.from_numpy(cr), torch.from_numpy(w)

    def grad_partial(self, iteration, member_begin, count, w_shard, sigma, out=None):
        acc = np.zeros(self.D, np.float64)
        for k in range(count):
            idx = self._idx(iteration, member_begin + k)
            acc += np.float64(w_shard[k].item()) * O.member_delta(self.table, idx, sigma, self.D,
                                                                  self.mutation).astype(np.float64)
        g = torch.from_numpy(acc.astype(np.float32))
        if out is not None:
            out.copy_(g)
            return out
        return g

    def grad_partial_range(self, iteration, member_begin, count, w_shard, sigma, j0, j1, out):
        g = self.grad_partial(iteration, member_begin, count, w_shard, sigma)
        out[j0:j1] = g[j0:j1]
        return out

    def adam_step(self, gsum, P, l2coeff, stepsize, beta1=0.9, beta2=0.999, epsilon=1e-08, sync=True):
        if self.adam is None:
            self.adam = O.AdamOracle(self.theta_src.copy(), stepsize, beta1, beta2, epsilon)
        self.adam.stepsize = stepsize                                      # stepsize_divisor changes it
        g = gsum.numpy().astype(np.float32) / np.float32(2 * P)
        ratio, theta = O.master_update(self.adam, g, l2coeff)
        self.theta32 = np.asarray(theta).astype(np.float32)
        self._ratio = float(ratio)
        return self._ratio if sync else None

    def last_ratio(self):
        return self._ratio


def tiny_workload(B=4, seed=0):
    import nicnes.synthetic as S
    dims = O.Dims(vocab_size=63, E=32, R=32, F=64)
    theta = O.make_theta(dims, seed, 4.0, 0.1)
    fc = np.random.Generator(np.random.PCG64(1234)).standard_normal((B, dims.F)).astype(np.float32)
    base, _, _ = O.decode(dims, theta, fc)
    gts, df, n = S.build_references(base, dims.vocab_size, seed=5, n_refs=5, df_sets=64)
    table = O.noise_table(1 << 16, 123)
    return dims, theta, fc, gts, df, n, table
