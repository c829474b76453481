"""CPU oracle for the NIC-NES population-evaluation path -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.
It is the checker, never the thing measured or shipped: the engine in
nes-img-captioning_amd/ never imports it.

Pieces and the reference lines they restate:
  noise table + index rule   new contract; replaces torch.normal_ in
                             PolicyNet.evolve, /root/reference/src/algorithm/nets.py:101-102
  perturb                    nets.py:113 (theta + delta, fp32) and
                             src/algorithm/nic_nes/nic_nes_worker.py:151 (theta - delta, fp32)
  decode                     oracle/nicnes_oracle.c (FCModel._sample, src/captioning/nets.py:183-245)
  fitness                    CaptPolicy.rollout 'greedy', src/captioning/policies.py:125 via
                             oracle/cider_ref.py
  compute_ranks / centered   NESMaster.compute_ranks / compute_centered_ranks,
                             src/algorithm/nic_nes/nic_nes_master.py:184-205 (stable tie-break)
  gradient                   NESMaster.gradient_estimate + batched_weighted_sum,
                             nic_nes_master.py:170-221 (fp64 accumulation, fp32 result)
  adam                       Adam.update/_compute_step, src/algorithm/nic_nes/optimizers.py:15-22,78-83
                             with g' = -g + l2coeff*theta, nic_nes_master.py:126,133

Pinned by tests/golden/ (made from the imported reference by scripts/make_golden.py), except
CIDEr-D whose reference implementation is absent (parity unpinned, see cider_ref.py).
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, 'libnicnes_oracle.so')
MASK64 = (1 << 64) - 1


# ------------------------------------------------------------------ C library ----------------
def build():
    subprocess.check_call(['make', '-s', '-C', HERE])


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        L.od_decode.restype = ctypes.c_int
        L.od_decode_sample.restype = ctypes.c_int
        L.od_param_count.restype = ctypes.c_int64
        _lib = L
    return _lib


class ODDims(ctypes.Structure):
    _fields_ = [('V1', ctypes.c_int32), ('E', ctypes.c_int32), ('R', ctypes.c_int32),
                ('F', ctypes.c_int32), ('T', ctypes.c_int32)]


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


# ------------------------------------------------------------------ model layout ------------
class Dims:
    """fc_caption dims; V1 = vocab_size + 1 (nets.py:151-152)."""

    def __init__(self, vocab_size=9487, E=128, R=128, F=2048, T=16):
        self.vocab_size, self.V1, self.E, self.R, self.F, self.T = vocab_size, vocab_size + 1, E, R, F, T

    def c(self):
        return ODDims(self.V1, self.E, self.R, self.F, self.T)

    def shapes(self):
        """(name, shape) in module registration order (nets.py:150-153, LSTMCore :81-82)."""
        V1, E, R, F = self.V1, self.E, self.R, self.F
        return [('img_embed.weight', (E, F)), ('img_embed.bias', (E,)),
                ('embed.weight', (V1, E)), ('logit.weight', (V1, R)), ('logit.bias', (V1,)),
                ('core.i2h.weight', (5 * R, E)), ('core.i2h.bias', (5 * R,)),
                ('core.h2h.weight', (5 * R, R)), ('core.h2h.bias', (5 * R,))]

    def offsets(self):
        out, o = {}, 0
        for name, shp in self.shapes():
            n = int(np.prod(shp))
            out[name] = (o, shp)
            o += n
        return out

    @property
    def D(self):
        return sum(int(np.prod(s)) for _, s in self.shapes())


def make_theta(dims, seed=0, gain=1.0, bias_std=0.0):
    """xavier_normal_ weights, zero (or N(0,bias_std)) biases, as PolicyNet.initialize_params
    (/root/reference/src/algorithm/nets.py:62-69) -- drawn from numpy PCG64(seed) so CPU and
    GPU boxes regenerate identical bits. gain > 1 gives the 'well-conditioned' fixtures."""
    rng = np.random.Generator(np.random.PCG64(seed))
    parts = []
    for name, shp in dims.shapes():
        if name.endswith('weight'):
            fan_out, fan_in = shp[0], shp[1]
            std = gain * np.sqrt(2.0 / float(fan_in + fan_out))
            parts.append((rng.standard_normal(shp) * std).astype(np.float32).ravel())
        else:
            if bias_std > 0:
                parts.append((rng.standard_normal(shp) * bias_std).astype(np.float32).ravel())
            else:
                parts.append(np.zeros(int(np.prod(shp)), np.float32))
    return np.concatenate(parts)


# ------------------------------------------------------------------ noise ------------------
def splitmix64(x):
    z = (x + 0x9E3779B97F4A7C15) & MASK64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK64
    return z ^ (z >> 31)


def noise_index(seed, iteration, member, table_len, dim):
    """include/nicnes_math.h nn_noise_index, restated with Python ints."""
    n_slots = (table_len - dim) // 64 + 1
    h = splitmix64((seed ^ (((iteration << 32) | (member & 0xffffffff)) & MASK64)) & MASK64)
    return (h % n_slots) * 64


def noise_table(table_len, seed=123):
    """The shared Gaussian table: numpy PCG64(seed) standard_normal float32."""
    return np.random.Generator(np.random.PCG64(seed)).standard_normal(table_len, dtype=np.float32)


def member_delta(table, idx, sigma, dim, mutation=None):
    """delta = fp32(sigma * z) (nets.py:102 draws N(0, sigma) in fp32), then the mutation transform
    of nets.py:104-112 in fp32: ('divide', s) -> delta / s (SM-G-SUM / SM-VECTOR), ('scale', a) ->
    delta * a (SM-PROPORTIONAL, a = |theta'|)."""
    delta = np.float32(sigma) * table[idx: idx + dim]
    if mutation is not None and mutation[0] != 'plain':
        mode, vec = mutation
        vec = np.asarray(vec, np.float32)
        delta = (delta / vec) if mode == 'divide' else (delta * vec)
    return delta.astype(np.float32)


def perturb(theta32, table, idx, sigma, sign, mutation=None):
    """theta +/- delta in fp32 (nets.py:113, nic_nes_worker.py:151)."""
    delta = member_delta(table, idx, sigma, theta32.size, mutation)
    return (theta32 + delta) if sign > 0 else (theta32 - delta)


# ------------------------------------------------------------------ decode -----------------
def decode(dims, theta32, fc, half_order=0):
    """Greedy decode of unique rows. Returns (seq int32 [B,T], lp f32 [B,T], fragile u8 [B,T])."""
    theta32 = np.ascontiguousarray(theta32, np.float32)
    fc = np.ascontiguousarray(fc, np.float32)
    B = fc.shape[0]
    assert theta32.size == dims.D and fc.shape[1] == dims.F
    seq = np.zeros((B, dims.T), np.int32)
    lp = np.zeros((B, dims.T), np.float32)
    fr = np.zeros((B, dims.T), np.uint8)
    d = dims.c()
    lib().od_decode(ctypes.byref(d), _p(theta32), _p(fc), ctypes.c_int(B), _p(seq), _p(lp), _p(fr),
                    ctypes.c_int(half_order))
    return seq, lp, fr


def decode_sample(dims, theta32, fc, u, half_order=0):
    """Sampled decode (FCModel._sample, greedy=False, nets.py:210-231) of B rows with the uniforms
    u [B, T] fp64 (row b's draw at logit step t in u[b, t-1]). Returns (seq, lp, fragile) as decode;
    fragile marks a draw within 1e-6 of a cdf boundary at the pick."""
    theta32 = np.ascontiguousarray(theta32, np.float32)
    fc = np.ascontiguousarray(fc, np.float32)
    B = fc.shape[0]
    u = np.ascontiguousarray(u, np.float64)
    assert theta32.size == dims.D and fc.shape[1] == dims.F and u.shape == (B, dims.T)
    seq = np.zeros((B, dims.T), np.int32)
    lp = np.zeros((B, dims.T), np.float32)
    fr = np.zeros((B, dims.T), np.uint8)
    d = dims.c()
    lib().od_decode_sample(ctypes.byref(d), _p(theta32), _p(fc), ctypes.c_int(B), _p(u), _p(seq), _p(lp), _p(fr),
                           ctypes.c_int(half_order))
    return seq, lp, fr


def gemv(W, bias, x, half_order=0):
    W = np.ascontiguousarray(W, np.float32)
    rows, K = W.shape
    out = np.zeros(rows, np.float32)
    lib().od_gemv(_p(W), _p(np.ascontiguousarray(bias, np.float32)), _p(np.ascontiguousarray(x, np.float32)),
                  ctypes.c_int(rows), ctypes.c_int(K), ctypes.c_int(half_order), _p(out))
    return out


def vec_math(which, x):
    x = np.ascontiguousarray(x, np.float32)
    out = np.empty_like(x)
    lib().od_vec_math(ctypes.c_int({'exp': 0, 'sigmoid': 1, 'tanh': 2}[which]), _p(x), _p(out),
                      ctypes.c_int64(x.size))
    return out


# ------------------------------------------------------------------ master side -------------
def compute_ranks(x):
    """nic_nes_master.py:196-205 with a STABLE argsort: ties ranked by position (the reference's
    default quicksort argsort leaves tie order implementation-defined)."""
    assert x.ndim == 1
    ranks = np.empty(len(x), dtype=int)
    ranks[x.argsort(kind='stable')] = np.arange(len(x))
    return ranks


def compute_centered_ranks(x):
    """nic_nes_master.py:184-194"""
    y = compute_ranks(x.ravel()).reshape(x.shape).astype(np.float64)
    y /= (x.size - 1)
    y -= .5
    return y


def weights_from_fitness(fitness):
    cr = compute_centered_ranks(np.asarray(fitness, np.float64))
    return (cr[:, 0] - cr[:, 1]).astype(np.float32), cr


def gradient(fitness, table, indices, sigma, dim, mutation=None):
    """nic_nes_master.py:170-182: g = sum_i w_i * delta_i / (2F). The engine accumulates in fp64
    in member order and rounds once to fp32 (the reference accumulates in fp32 BLAS order)."""
    w, _ = weights_from_fitness(fitness)
    acc = np.zeros(dim, np.float64)
    for i, idx in enumerate(indices):
        delta = member_delta(table, int(idx), sigma, dim, mutation)
        acc += np.float64(w[i]) * delta.astype(np.float64)
    g = acc.astype(np.float32)
    g /= np.float32(2 * len(indices))
    return g


class AdamOracle:
    """optimizers.py:15-22,78-83 with fp64 state; update() takes the reference's globalg."""

    def __init__(self, theta, stepsize, beta1=0.9, beta2=0.999, epsilon=1e-08):
        self.theta = theta
        self.dim = len(theta)
        self.t = 0
        self.stepsize, self.beta1, self.beta2, self.epsilon = stepsize, beta1, beta2, epsilon
        self.m = np.zeros(self.dim, dtype=np.float64)
        self.v = np.zeros(self.dim, dtype=np.float64)

    def update(self, globalg):
        self.t += 1
        a = self.stepsize * np.sqrt(1 - self.beta2 ** self.t) / (1 - self.beta1 ** self.t)
        self.m = self.beta1 * self.m + (1 - self.beta1) * globalg
        self.v = self.beta2 * self.v + (1 - self.beta2) * (globalg * globalg)
        step = -a * self.m / (np.sqrt(self.v) + self.epsilon)
        ratio = np.linalg.norm(step) / np.linalg.norm(self.theta)
        self.theta = self.theta + step
        return ratio, self.theta


class SGDOracle:
    """optimizers.py:38-47 (SGD with momentum), fp64 state."""

    def __init__(self, theta, stepsize, momentum=0.9):
        self.theta = theta
        self.dim = len(theta)
        self.t = 0
        self.stepsize, self.momentum = stepsize, momentum
        self.v = np.zeros(self.dim, dtype=np.float64)

    def update(self, globalg):
        self.t += 1
        self.v = self.momentum * self.v + (1. - self.momentum) * globalg
        step = -self.stepsize * self.v
        ratio = np.linalg.norm(step) / np.linalg.norm(self.theta)
        self.theta = self.theta + step
        return ratio, self.theta


def master_update(adam, g, l2coeff):
    """nic_nes_master.py:126-133: reg = l2coeff * theta (theta fp32 before the first update,
    fp64 after: fact 8 of SURVEY.md), globalg = -g + reg."""
    reg = l2coeff * adam.theta   # python float * fp32 array stays fp32 (NEP 50), fp64 after step 1
    return adam.update(-g + reg)
