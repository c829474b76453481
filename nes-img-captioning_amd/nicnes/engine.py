"""Engine: a Python owner of one libnicnes handle on one GPU.

PyTorch-ROCm tensors are used for device storage only (their data_ptr() goes through the C ABI);
all arithmetic of the path runs in the HIP kernels of libnicnes.so.
"""
import ctypes
import os

import numpy as np
import torch

from . import _lib
from ._lib import NicnesConfig, check

SEQ_LENGTH = 16          # FCModel.seq_length, /root/reference/src/captioning/nets.py:147


def pack_ngram(tokens):
    """Exact uint64 key of an n-gram of token ids (n<<56 | t0<<42 | t1<<28 | t2<<14 | t3); the
    word strings of array_to_str (/root/reference/src/algorithm/tools/utils.py:34-40) are the ids."""
    n = len(tokens)
    assert 1 <= n <= 4
    key = n << 56
    for k, t in enumerate(tokens):
        t = int(t)
        assert 0 <= t < 16384
        key |= t << (42 - 14 * k)
    return key


def df_table_arrays(document_frequency):
    """{tuple-of-str-or-int n-gram: df} -> (sorted uint64 keys, float64 df)."""
    items = sorted((pack_ngram(tuple(int(w) for w in g)), float(v)) for g, v in document_frequency.items())
    keys = np.array([k for k, _ in items], dtype=np.uint64)
    vals = np.array([v for _, v in items], dtype=np.float64)
    return keys, vals


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


class Engine:
    """One handle = one GPU. ``device`` is the local cuda index."""

    def __init__(self, vocab_size=9487, input_encoding_size=128, rnn_size=128, fc_feat_size=2048,  # noqa: E501
                 seq_length=SEQ_LENGTH, max_batch=128, max_refs=None, max_members=512, noise_len=1 << 27,
                 noise_seed=0, device=0, lib_path=None):
        self.L = _lib.lib(lib_path)
        self.device = torch.device('cuda', device)
        self.cfg = NicnesConfig(vocab_size, input_encoding_size, rnn_size, fc_feat_size, seq_length, max_batch,
                                max_refs or 8 * max_batch, max_members, noise_len, noise_seed)
        self.D = int(self.L.nicnes_param_count(ctypes.byref(self.cfg)))
        off = (ctypes.c_int64 * 10)()
        check(self.L.nicnes_param_offsets(ctypes.byref(self.cfg), off), None, 'nicnes_param_offsets')
        self.offsets = list(off)
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            check(self.L.nicnes_create(ctypes.byref(self.cfg), device, ctypes.byref(h)), None, 'nicnes_create')
        self.h = h
        self.n_cu = torch.cuda.get_device_properties(self.device).multi_processor_count
        self.coop_mode = 0 if os.environ.get('NICNES_DECODE_COOP') == '0' else 1
        self._keep = {}
        self.B = 0
        self.fitness_mode = 0
        self.rpi = 1

    # -------------------------------------------------------------------------------------
    def close(self):
        if getattr(self, 'h', None):
            self.L.nicnes_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def _dev(self, a, dtype):
        if isinstance(a, torch.Tensor):
            return a.to(device=self.device, dtype=dtype).contiguous()
        return torch.from_numpy(np.ascontiguousarray(a)).to(device=self.device, dtype=dtype)

    # ---------------------------------------------------------------- state -------------
    def set_noise_table(self, table):
        t = self._dev(table, torch.float32)
        assert t.numel() == self.cfg.noise_len
        self._keep['noise'] = t
        check(self.L.nicnes_set_noise_table(self.h, _ptr(t), ctypes.c_uint64(t.numel())), self.h, 'set_noise_table')

    def set_theta(self, theta, fp32_origin=None):
        """theta: fp32 (reference start, fp32 first-step semantics) or fp64 vector [D]."""
        if fp32_origin is None:
            fp32_origin = (theta.dtype == np.float32) if isinstance(theta, np.ndarray) else theta.dtype == torch.float32
        t = self._dev(theta, torch.float64)
        assert t.numel() == self.D
        with torch.cuda.device(self.device):
            check(self.L.nicnes_set_theta(self.h, _ptr(t), int(bool(fp32_origin)), self._stream()), self.h, 'set_theta')
        self._keep['theta_in'] = t

    def theta(self):
        t64 = torch.empty(self.D, dtype=torch.float64, device=self.device)
        t32 = torch.empty(self.D, dtype=torch.float32, device=self.device)
        with torch.cuda.device(self.device):
            check(self.L.nicnes_get_theta(self.h, _ptr(t64), _ptr(t32), self._stream()), self.h, 'get_theta')
        return t64, t32

    def adam_state(self):
        m = torch.empty(self.D, dtype=torch.float64, device=self.device)
        v = torch.empty(self.D, dtype=torch.float64, device=self.device)
        t = ctypes.c_int64()
        with torch.cuda.device(self.device):
            check(self.L.nicnes_get_adam_state(self.h, _ptr(m), _ptr(v), ctypes.byref(t), self._stream()), self.h,
                  'get_adam_state')
        return m, v, t.value

    def set_adam_state(self, m, v, t):
        m = self._dev(m, torch.float64)
        v = self._dev(v, torch.float64)
        with torch.cuda.device(self.device):
            check(self.L.nicnes_set_adam_state(self.h, _ptr(m), _ptr(v), int(t), self._stream()), self.h,
                  'set_adam_state')
        self._keep['adam_m'], self._keep['adam_v'] = m, v

    def set_df_table(self, keys, df, ref_len_log):
        k = self._dev(np.asarray(keys, np.uint64).view(np.int64), torch.int64)
        d = self._dev(np.asarray(df, np.float64), torch.float64)
        self._keep['df_keys'], self._keep['df_vals'] = k, d
        check(self.L.nicnes_set_df_table(self.h, _ptr(k), _ptr(d), int(k.numel()), float(ref_len_log)), self.h,
              'set_df_table')

    def set_batch(self, fc, gts):
        """fc [B, F] fp32 of unique images; gts: per image an int array [n_i, seq_length] of
        zero-padded label rows (data['gts'], /root/reference/src/captioning/dataloader.py:162)."""
        self.set_batches([(fc, gts)])

    def set_batches(self, batches):
        """Several batches of equal size B at once, [(fc [B, F], gts), ...], for per-member batches
        (single_batch: false, /root/reference/src/algorithm/nic_nes/nic_nes_worker.py:121-128): an
        evaluate's member_batch then names each member's batch."""
        fcs, rows, start = [], [], [0]
        for fc, gts in batches:
            fc_np = fc.detach().cpu().numpy() if isinstance(fc, torch.Tensor) else np.asarray(fc, np.float32)
            if len(gts) != fc_np.shape[0]:
                raise ValueError('gts has %d images, fc has %d rows' % (len(gts), fc_np.shape[0]))
            fcs.append(np.asarray(fc_np, np.float32))
            for g in gts:
                g = np.asarray(g, np.int32).reshape(-1, self.cfg.seq_length)
                rows.append(g)
                start.append(start[-1] + g.shape[0])
        B = fcs[0].shape[0]
        if any(f.shape[0] != B for f in fcs):
            raise ValueError('batches must have the same number of images')
        fc_t = self._dev(np.concatenate(fcs, 0), torch.float32)
        refs = self._dev(np.concatenate(rows, 0), torch.int32)
        starts = self._dev(np.array(start, np.int32), torch.int32)
        self._keep['fc'], self._keep['refs'], self._keep['ref_start'] = fc_t, refs, starts
        with torch.cuda.device(self.device):
            check(self.L.nicnes_set_batches(self.h, _ptr(fc_t), len(fcs), B, _ptr(refs), int(refs.shape[0]),
                                            _ptr(starts), self._stream()), self.h, 'set_batches')
        self.B = B
        self.n_batches = len(fcs)

    # ---------------------------------------------------------------- the hot path -------
    def noise_indices(self, iteration, member_begin, count):
        out = torch.empty(count, dtype=torch.int64, device=self.device)
        with torch.cuda.device(self.device):
            check(self.L.nicnes_noise_indices(self.h, ctypes.c_uint64(iteration), member_begin, count, _ptr(out),
                                              self._stream()), self.h, 'noise_indices')
        return out

    def noise_vectors(self, iteration, member_begin, count, sigma, out=None):
        """delta [count, D] fp32 = fp32(sigma * table slice) of members [member_begin, +count) (the
        vectors a reference-format NESResult carries)."""
        o = out if out is not None else torch.empty((count, self.D), dtype=torch.float32, device=self.device)
        with torch.cuda.device(self.device):
            check(self.L.nicnes_noise_vectors(self.h, ctypes.c_uint64(iteration), member_begin, count,
                                              ctypes.c_float(sigma), _ptr(o), self._stream()), self.h, 'noise_vectors')
        return o

    MUTATION_MODES = {'plain': 0, 'divide': 1, 'scale': 2}

    def set_mutation(self, mode='plain', vec=None):
        """Per-parameter noise transform of safe / proportional mutations: 'divide' (delta / vec:
        SM-G-SUM, SM-G-ABS, SM-VECTOR with vec = the sensitivity), 'scale' (delta * vec:
        SM-PROPORTIONAL), 'plain' off."""
        code = self.MUTATION_MODES[mode] if isinstance(mode, str) else int(mode)
        v = self._dev(vec, torch.float32) if vec is not None else None
        if v is not None and v.numel() != self.D:
            raise ValueError('mutation vector needs D entries')
        with torch.cuda.device(self.device):
            check(self.L.nicnes_set_mutation(self.h, code, _ptr(v), self._stream()), self.h, 'set_mutation')
        self._keep['mutation'] = v
        self.mutation_mode = code

    def set_mutation_proportional(self, mean_abs):
        """SM-PROPORTIONAL's vector formed on the device from the handle's fp32 theta
        (nicnes_set_mutation_proportional): |theta| with exact zeros replaced by mean_abs, the caller's fp32
        mean of |theta| (nets.py:108-112); then mode 'scale'."""
        with torch.cuda.device(self.device):
            check(self.L.nicnes_set_mutation_proportional(self.h, float(mean_abs), self._stream()), self.h,
                  'set_mutation_proportional')
        self._keep['mutation'] = None
        self.mutation_mode = self.MUTATION_MODES['scale']

    def theta_zeros(self):
        """How many entries of the fp32 theta are exactly zero (nicnes_theta_zeros; synchronises)."""
        out = ctypes.c_int64(0)
        with torch.cuda.device(self.device):
            check(self.L.nicnes_theta_zeros(self.h, ctypes.byref(out), self._stream()), self.h, 'theta_zeros')
        return int(out.value)

    # Fitness enum values the engine implements (src/captioning/policies.py:22-35) -> nicnes.h codes
    FITNESS_MODES = {'greedy': 0, 'greedy_logprob': 1, 'greedy_expprob': 2, 'greedy_linprob': 3,
                     'greedy_avgprob': 4, 'sample': 5, 'self_critical': 6, 'sc_loss': 7}
    SAMPLED_MODES = (5, 6, 7)

    def set_fitness_mode(self, fitness):
        """Fitness criterion by its experiment-JSON name (policy_options.fitness) or nicnes.h code."""
        code = self.FITNESS_MODES.get(fitness, fitness) if isinstance(fitness, str) else int(fitness)
        if isinstance(code, str):
            code = -1
        check(self.L.nicnes_set_fitness_mode(self.h, code), self.h, 'set_fitness_mode(%r)' % (fitness,))
        self.fitness_mode = code

    def evaluate(self, iteration, member_begin, count, sigma, fitness_out=None, return_seq=False, return_lp=False,
                 member_batch=None):
        """Fitness (f+, f-) of members [member_begin, +count): tensor [count, 2] fp64 on the GPU.
        return_seq / return_lp add the greedy tokens [count, 2, B, T] int32 and their per-step
        log-probs (FCModel._sample's seq_logprobs) [count, 2, B, T] fp32. member_batch: per member the
        index of its batch among set_batches' (None: the one batch held)."""
        fit = fitness_out if fitness_out is not None else torch.empty((count, 2), dtype=torch.float64,
                                                                      device=self.device)
        shape = (count, 2, self.rollout_rows(), self.cfg.seq_length)
        seq = torch.empty(shape, dtype=torch.int32, device=self.device) if return_seq else None
        lp = torch.empty(shape, dtype=torch.float32, device=self.device) if return_lp else None
        mb = None
        if member_batch is not None:
            mb_np = np.ascontiguousarray(np.asarray(member_batch, np.int32))
            if mb_np.shape != (count,):
                raise ValueError('member_batch needs one entry per member')
            mb = mb_np.ctypes.data_as(ctypes.c_void_p)
        with torch.cuda.device(self.device):
            check(self.L.nicnes_evaluate_batches(self.h, ctypes.c_uint64(iteration), member_begin, count,
                                                 ctypes.c_float(sigma), mb, _ptr(fit), _ptr(seq), _ptr(lp),
                                                 self._stream()), self.h, 'evaluate')
        out = (fit,) + ((seq,) if return_seq else ()) + ((lp,) if return_lp else ())
        return out if len(out) > 1 else fit

    def set_rows_per_image(self, n=1):
        """Sampled modes: decode n rows per image of the batch (the reference's seq_per_img copies, each with
        its own draws); greedy modes always decode one."""
        check(self.L.nicnes_set_rows_per_image(self.h, int(n)), self.h, 'set_rows_per_image')
        self.rpi = int(n)

    def rollout_rows(self):
        """Rows of one rollout: the batch's images, times rows_per_image in the sampled modes."""
        return self.B * (getattr(self, 'rpi', 1) if self.fitness_mode in self.SAMPLED_MODES else 1)

    def set_sample_draws(self, u=None):
        """Test hook: the uniforms [count, 2, B, T] fp64 the next sampled evaluates use (None: the engine's
        own counter-based draws)."""
        if u is None:
            check(self.L.nicnes_set_sample_draws(self.h, None, 0), self.h, 'set_sample_draws')
            self._keep.pop('draws', None)
            return
        a = np.ascontiguousarray(np.asarray(u, np.float64))
        check(self.L.nicnes_set_sample_draws(self.h, a.ctypes.data_as(ctypes.c_void_p), a.size), self.h,
              'set_sample_draws')
        self._keep['draws'] = a

    def evaluate_theta(self, batch=0, return_seq=False, return_lp=False, iteration=0):
        """Fitness of theta itself on the batch held (or batch `batch` of set_batches'): the sigma = 0
        rollout (CaptPolicy.rollout) decoded once, sign + over the first half of the images and sign -
        over the rest. Tensor [1] fp64 on the GPU; return_seq / return_lp add [B, T] tokens / log-probs.
        iteration: the draw stream of the sampled modes (each eval rollout its own)."""
        fit = torch.empty(1, dtype=torch.float64, device=self.device)
        shape = (self.rollout_rows(), self.cfg.seq_length)
        seq = torch.empty(shape, dtype=torch.int32, device=self.device) if return_seq else None
        lp = torch.empty(shape, dtype=torch.float32, device=self.device) if return_lp else None
        with torch.cuda.device(self.device):
            check(self.L.nicnes_evaluate_theta(self.h, int(batch), int(iteration), _ptr(fit), _ptr(seq), _ptr(lp),
                                               self._stream()),
                  self.h, 'evaluate_theta')
        out = (fit,) + ((seq,) if return_seq else ()) + ((lp,) if return_lp else ())
        return out if len(out) > 1 else fit

    def rank_weights(self, fitness_all):
        """fitness [P, 2] fp64 (whole population) -> (centred ranks [P, 2] fp64, weights [P] fp32)."""
        P = fitness_all.shape[0]
        cr = torch.empty((P, 2), dtype=torch.float64, device=self.device)
        w = torch.empty(P, dtype=torch.float32, device=self.device)
        with torch.cuda.device(self.device):
            check(self.L.nicnes_rank_weights(self.h, _ptr(fitness_all), P, _ptr(cr), _ptr(w), self._stream()), self.h,
                  'rank_weights')
        return cr, w

    def grad_partial(self, iteration, member_begin, count, w_shard, sigma, out=None):
        g = out if out is not None else torch.empty(self.D, dtype=torch.float32, device=self.device)
        with torch.cuda.device(self.device):
            check(self.L.nicnes_grad_partial(self.h, ctypes.c_uint64(iteration), member_begin, count, _ptr(w_shard),
                                             ctypes.c_float(sigma), _ptr(g), self._stream()), self.h, 'grad_partial')
        return g

    def grad_partial_range(self, iteration, member_begin, count, w_shard, sigma, j0, j1, out):
        """grad_partial on parameters [j0, j1) of `out` (j0 a multiple of 64)."""
        with torch.cuda.device(self.device):
            check(self.L.nicnes_grad_partial_range(self.h, ctypes.c_uint64(iteration), member_begin, count,
                                                   _ptr(w_shard), ctypes.c_float(sigma), int(j0), int(j1), _ptr(out),
                                                   self._stream()), self.h, 'grad_partial_range')
        return out

    def adam_step(self, gsum, P, l2coeff, stepsize, beta1=0.9, beta2=0.999, epsilon=1e-08, sync=True):
        """Adam on the engine's theta. sync=True returns the update ratio (one host sync); sync=False
        only enqueues the step and returns None (read the ratio later with last_ratio())."""
        ratio = ctypes.c_double()
        with torch.cuda.device(self.device):
            check(self.L.nicnes_adam_step(self.h, _ptr(gsum), P, l2coeff, stepsize, beta1, beta2, epsilon,
                                          ctypes.byref(ratio) if sync else None, self._stream()), self.h, 'adam_step')
        return ratio.value if sync else None

    def last_ratio(self):
        """Update ratio of the newest optimizer step (synchronising)."""
        ratio = ctypes.c_double()
        with torch.cuda.device(self.device):
            check(self.L.nicnes_last_ratio(self.h, ctypes.byref(ratio), self._stream()), self.h, 'last_ratio')
        return ratio.value

    def sgd_step(self, gsum, P, l2coeff, stepsize, momentum=0.9):
        ratio = ctypes.c_double()
        with torch.cuda.device(self.device):
            check(self.L.nicnes_sgd_step(self.h, _ptr(gsum), P, l2coeff, stepsize, momentum, ctypes.byref(ratio),
                                         self._stream()), self.h, 'sgd_step')
        return ratio.value

    def optimizer_update(self, globalg, kind='adam', stepsize=1e-3, beta1=0.9, beta2=0.999, epsilon=1e-08):
        """Optimizer.update(globalg) form: globalg [D] fp32 or fp64 -> update ratio."""
        is32 = (globalg.dtype == torch.float32) if isinstance(globalg, torch.Tensor) else \
            (np.asarray(globalg).dtype == np.float32)
        g = self._dev(globalg, torch.float64)
        ratio = ctypes.c_double()
        with torch.cuda.device(self.device):
            check(self.L.nicnes_optimizer_update(self.h, {'adam': 0, 'sgd': 1}[kind], _ptr(g), int(is32), stepsize,
                                                 beta1, beta2, epsilon, ctypes.byref(ratio), self._stream()), self.h,
                  'optimizer_update')
        return ratio.value

    def set_timing(self, on=True):
        check(self.L.nicnes_set_timing(self.h, int(bool(on))), self.h, 'set_timing')

    def kernel_times(self):
        """(decode_ms, cider_ms) of the last evaluate() (HIP events on its stream)."""
        out = (ctypes.c_float * 2)()
        check(self.L.nicnes_kernel_times(self.h, out), self.h, 'kernel_times')
        return float(out[0]), float(out[1])

    def decode_phase_times(self):
        """Per-kernel split of the last timed decode (HIP events between its launches): img_ms,
        step_ms / step_launches (fused path: the steps kernel, every step t = -1..T in one launch; one
        launch per step in DECODE_PROF timing builds, whose first two, cell-only, launches are also in
        cell_only_ms), logit_ms / logit_launches and cell_ms / cell_launches (split path)."""
        out = (ctypes.c_float * 8)()
        check(self.L.nicnes_decode_phase_times(self.h, out), self.h, 'decode_phase_times')
        return {'img_ms': float(out[0]), 'cell_only_ms': float(out[1]), 'step_ms': float(out[2]),
                'step_launches': int(out[3]), 'logit_ms': float(out[4]), 'logit_launches': int(out[5]),
                'cell_ms': float(out[6]), 'cell_launches': int(out[7])}

    def set_decode_split(self, S=0, G=0):
        """Force the decode shape (S logit workgroups per member slab, G = 4 / 2 row groups per slab);
        0 = automatic. Tokens do not depend on it."""
        check(self.L.nicnes_set_decode_split(self.h, int(S), int(G)), self.h, 'set_decode_split')

    def set_decode_streams(self, n=0):
        """Split the evaluate's members over n streams (0 = automatic: 2 on the split path, 1 fused).
        Tokens do not depend on it."""
        check(self.L.nicnes_set_decode_streams(self.h, int(n)), self.h, 'set_decode_streams')

    def sum_sensitivity(self, rows, underflow=0.0, out=None):
        """SM-G-SUM sensitivity (Sensitivity.calc_sensitivity, safe_mutations.py:34-117) of the current theta
        on the first `rows` images of the batch held: fp32 [D] on the GPU, clamped and scaled by
        `underflow` when it is > 0 (the vector set_mutation('divide', ...) takes)."""
        v = out if out is not None else torch.empty(self.D, dtype=torch.float32, device=self.device)
        with torch.cuda.device(self.device):
            check(self.L.nicnes_sum_sensitivity(self.h, int(rows), ctypes.c_float(underflow), _ptr(v), self._stream()),
                  self.h, 'sum_sensitivity')
        return v

    def set_decode_coop(self, mode=1):
        """1 (default): the split shape (128-row slabs, S = 2 or 4, every workgroup resident) runs as one
        persistent launch whose workgroups hand partial states and h' to each other; 0: two launches per
        step. Tokens do not depend on it."""
        check(self.L.nicnes_set_decode_coop(self.h, int(mode)), self.h, 'set_decode_coop')
        self.coop_mode = int(mode)

    def last_decode_bounded(self):
        """True when the last greedy decode enqueued used the pair-bounded lse (the steps kernel's PAIRS instantiation)."""
        out = ctypes.c_int32()
        check(self.L.nicnes_last_decode_lse(self.h, ctypes.byref(out)), self.h, 'last_decode_lse')
        return bool(out.value)

    def decode_path(self, B=None, count=1):
        """'fused', 'split' or 'coop': the decode path an evaluate of `count` members would take."""
        out = ctypes.c_int32()
        check(self.L.nicnes_decode_path(self.h, int(B or self.B), int(count), ctypes.byref(out)), self.h, 'decode_path')
        return ('fused', 'split', 'coop')[out.value]

    def decode_shape(self, B=None, count=1):
        """(G, slabs, S) an evaluate of `count` members would use."""
        out = (ctypes.c_int32 * 3)()
        check(self.L.nicnes_decode_shape(self.h, int(B or self.B), int(count), out), self.h, 'decode_shape')
        return tuple(int(v) for v in out)

    # ---------------------------------------------------------------- multi-GPU (RCCL) ----------
    @staticmethod
    def comm_unique_id():
        """128-byte RCCL id, made by rank 0 and sent to the other ranks out of band."""
        buf = (ctypes.c_uint8 * _lib.COMM_ID_BYTES)()
        check(_lib.lib().nicnes_comm_unique_id(buf), None, 'comm_unique_id')
        return bytes(buf)

    def comm_init(self, nranks, rank, uid):
        """Join the RCCL communicator `uid` as `rank` of `nranks` (collective over the ranks)."""
        buf = (ctypes.c_uint8 * _lib.COMM_ID_BYTES).from_buffer_copy(uid)
        with torch.cuda.device(self.device):
            check(self.L.nicnes_comm_init(self.h, int(nranks), int(rank), buf), self.h, 'comm_init')
        self.comm_ranks = int(nranks)

    def comm_destroy(self):
        check(self.L.nicnes_comm_destroy(self.h), self.h, 'comm_destroy')
        self.comm_ranks = 1

    def comm_count(self):
        """(ranks, this rank) as RCCL reports them for the bound communicator ((1, 0) with none)."""
        n, r = ctypes.c_int32(), ctypes.c_int32()
        check(self.L.nicnes_comm_count(self.h, ctypes.byref(n), ctypes.byref(r)), self.h, 'comm_count')
        return int(n.value), int(r.value)

    def allgather_fitness(self, fit_local, fit_all):
        """fit_all [P_local * nranks, 2] <- every rank's fit_local [P_local, 2] (rank order)."""
        with torch.cuda.device(self.device):
            check(self.L.nicnes_allgather_fitness(self.h, _ptr(fit_local), int(fit_local.shape[0]), _ptr(fit_all),
                                                  self._stream()), self.h, 'allgather_fitness')
        return fit_all

    def allreduce_grad(self, gsum):
        """gsum [D] fp32 summed in place over the ranks."""
        with torch.cuda.device(self.device):
            check(self.L.nicnes_allreduce_grad(self.h, _ptr(gsum), self._stream()), self.h, 'allreduce_grad')
        return gsum

    def clear_faults(self):
        """Clear a contained decode fault (nicnes_clear_faults): returns the fault counters it found
        {'coop_timeouts', 'sample_slot_timeouts'}; the handle evaluates again afterwards."""
        out = (ctypes.c_int64 * 2)()
        with torch.cuda.device(self.device):
            check(self.L.nicnes_clear_faults(self.h, out), self.h, 'clear_faults')
        return {'coop_timeouts': int(out[0]), 'sample_slot_timeouts': int(out[1])}

    def stats(self):
        out = (ctypes.c_int64 * 4)()
        check(self.L.nicnes_stats(self.h, out), self.h, 'stats')
        return {'tie_fallbacks': out[0], 'sample_stage_fallbacks': out[1], 'coop_timeouts': out[2],
                'sample_slot_timeouts': out[3]}
