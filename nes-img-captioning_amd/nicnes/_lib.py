"""ctypes binding of libnicnes.so (include/nicnes.h). No fallback: a missing library is an error."""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, 'libnicnes.so')

OK, ERR_INVALID, ERR_UNSUPPORTED, ERR_HIP, ERR_NOMEM, ERR_FAULT = 0, 1, 2, 3, 4, 5
COMM_ID_BYTES = 128
_NAMES = {ERR_INVALID: 'invalid argument', ERR_UNSUPPORTED: 'not supported', ERR_HIP: 'HIP error',
          ERR_NOMEM: 'out of device memory', ERR_FAULT: 'contained decode fault'}

# every symbol include/nicnes.h declares (checked by tests/test_abi.py)
EXPORTS = ['nicnes_param_count', 'nicnes_param_offsets', 'nicnes_create', 'nicnes_destroy', 'nicnes_last_error',
           'nicnes_set_noise_table', 'nicnes_set_theta', 'nicnes_get_theta', 'nicnes_set_adam_state',
           'nicnes_get_adam_state', 'nicnes_set_batch', 'nicnes_set_df_table', 'nicnes_noise_indices',
           'nicnes_evaluate', 'nicnes_rank_weights', 'nicnes_grad_partial', 'nicnes_adam_step', 'nicnes_stats',
           'nicnes_set_timing', 'nicnes_kernel_times', 'nicnes_decode_phase_times', 'nicnes_sgd_step',
           'nicnes_optimizer_update', 'nicnes_last_ratio', 'nicnes_set_fitness_mode', 'nicnes_evaluate_lp',
           'nicnes_set_decode_split', 'nicnes_decode_shape', 'nicnes_set_decode_streams', 'nicnes_comm_unique_id', 'nicnes_comm_init',
           'nicnes_comm_attach', 'nicnes_comm_destroy', 'nicnes_comm_count', 'nicnes_clear_faults', 'nicnes_allgather_fitness', 'nicnes_allreduce_grad',
           'nicnes_noise_vectors', 'nicnes_set_batches', 'nicnes_evaluate_batches', 'nicnes_set_mutation',
           'nicnes_set_mutation_proportional', 'nicnes_theta_zeros',
           'nicnes_set_decode_coop', 'nicnes_decode_path', 'nicnes_sum_sensitivity', 'nicnes_grad_partial_range',
           'nicnes_evaluate_theta', 'nicnes_set_sample_draws', 'nicnes_set_rows_per_image',
           'nicnes_last_decode_lse']


class NicnesConfig(ctypes.Structure):
    _fields_ = [('vocab_size', ctypes.c_int32), ('input_encoding_size', ctypes.c_int32),
                ('rnn_size', ctypes.c_int32), ('fc_feat_size', ctypes.c_int32), ('seq_length', ctypes.c_int32),
                ('max_batch', ctypes.c_int32), ('max_refs', ctypes.c_int32), ('max_members', ctypes.c_int32),
                ('noise_len', ctypes.c_uint64), ('noise_seed', ctypes.c_uint64)]


class NicnesError(RuntimeError):
    pass


class DecodeFault(NicnesError):
    """NICNES_ERR_FAULT: a decode lost rows (coop hand-off or logit-slot timeout); the iteration's fitness is
    NaN and its optimizer step was skipped on every rank, so theta / m / v are those before it.
    Engine.clear_faults() makes the handle usable again."""


_libs = {}


def lib(path=None):
    """Load the in-tree engine library (built by `make -C nes-img-captioning_amd`). `path` selects
    another build of the same ABI (timing-only variants, scripts/ablate.py)."""
    path = path or LIB_PATH
    if path in _libs:
        return _libs[path]
    if not os.path.exists(path):
        raise NicnesError('%s not built: run `make -C nes-img-captioning_amd` '
                          '(or __graft_entry__.build()); there is no CPU fallback' % os.path.basename(path))
    L = ctypes.CDLL(path)
    c = ctypes
    vp, i32, i64, u64, f32, f64 = c.c_void_p, c.c_int32, c.c_int64, c.c_uint64, c.c_float, c.c_double
    sig = {
        'nicnes_param_count': (i64, [vp]),
        'nicnes_param_offsets': (c.c_int, [vp, vp]),
        'nicnes_create': (c.c_int, [vp, c.c_int, c.POINTER(vp)]),
        'nicnes_destroy': (c.c_int, [vp]),
        'nicnes_last_error': (c.c_char_p, [vp]),
        'nicnes_set_noise_table': (c.c_int, [vp, vp, u64]),
        'nicnes_set_theta': (c.c_int, [vp, vp, c.c_int, vp]),
        'nicnes_get_theta': (c.c_int, [vp, vp, vp, vp]),
        'nicnes_set_adam_state': (c.c_int, [vp, vp, vp, i64, vp]),
        'nicnes_get_adam_state': (c.c_int, [vp, vp, vp, vp, vp]),
        'nicnes_set_batch': (c.c_int, [vp, vp, i32, vp, i32, vp, vp]),
        'nicnes_set_df_table': (c.c_int, [vp, vp, vp, i64, f64]),
        'nicnes_noise_indices': (c.c_int, [vp, u64, i32, i32, vp, vp]),
        'nicnes_evaluate': (c.c_int, [vp, u64, i32, i32, f32, vp, vp, vp]),
        'nicnes_evaluate_lp': (c.c_int, [vp, u64, i32, i32, f32, vp, vp, vp, vp]),
        'nicnes_set_fitness_mode': (c.c_int, [vp, i32]),
        'nicnes_noise_vectors': (c.c_int, [vp, u64, i32, i32, f32, vp, vp]),
        'nicnes_set_batches': (c.c_int, [vp, vp, i32, i32, vp, i32, vp, vp]),
        'nicnes_set_mutation': (c.c_int, [vp, i32, vp, vp]),
        'nicnes_set_mutation_proportional': (c.c_int, [vp, c.c_float, vp]),
        'nicnes_theta_zeros': (c.c_int, [vp, vp, vp]),
        'nicnes_evaluate_batches': (c.c_int, [vp, u64, i32, i32, f32, vp, vp, vp, vp, vp]),
        'nicnes_evaluate_theta': (c.c_int, [vp, i32, u64, vp, vp, vp, vp]),
        'nicnes_set_sample_draws': (c.c_int, [vp, vp, i64]),
        'nicnes_set_rows_per_image': (c.c_int, [vp, i32]),
        'nicnes_rank_weights': (c.c_int, [vp, vp, i32, vp, vp, vp]),
        'nicnes_grad_partial': (c.c_int, [vp, u64, i32, i32, vp, f32, vp, vp]),
        'nicnes_grad_partial_range': (c.c_int, [vp, u64, i32, i32, vp, f32, i64, i64, vp, vp]),
        'nicnes_adam_step': (c.c_int, [vp, vp, i32, f64, f64, f64, f64, f64, vp, vp]),
        'nicnes_stats': (c.c_int, [vp, vp]),
        'nicnes_set_timing': (c.c_int, [vp, c.c_int]),
        'nicnes_kernel_times': (c.c_int, [vp, vp]),
        'nicnes_decode_phase_times': (c.c_int, [vp, vp]),
        'nicnes_set_decode_split': (c.c_int, [vp, i32, i32]),
        'nicnes_decode_shape': (c.c_int, [vp, i32, i32, vp]),
        'nicnes_set_decode_streams': (c.c_int, [vp, i32]),
        'nicnes_set_decode_coop': (c.c_int, [vp, i32]),
        'nicnes_decode_path': (c.c_int, [vp, i32, i32, vp]),
        'nicnes_last_decode_lse': (c.c_int, [vp, vp]),
        'nicnes_sum_sensitivity': (c.c_int, [vp, i32, f32, vp, vp]),
        'nicnes_comm_unique_id': (c.c_int, [vp]),
        'nicnes_comm_init': (c.c_int, [vp, i32, i32, vp]),
        'nicnes_comm_attach': (c.c_int, [vp, vp]),
        'nicnes_comm_destroy': (c.c_int, [vp]),
        'nicnes_comm_count': (c.c_int, [vp, vp, vp]),
        'nicnes_clear_faults': (c.c_int, [vp, vp]),
        'nicnes_allgather_fitness': (c.c_int, [vp, vp, i32, vp, vp]),
        'nicnes_allreduce_grad': (c.c_int, [vp, vp, vp]),
        'nicnes_last_ratio': (c.c_int, [vp, vp, vp]),
        'nicnes_sgd_step': (c.c_int, [vp, vp, i32, f64, f64, f64, vp, vp]),
        'nicnes_optimizer_update': (c.c_int, [vp, c.c_int, vp, c.c_int, f64, f64, f64, f64, vp, vp]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _libs[path] = L
    return L


def check(rc, handle=None, what=''):
    if rc != OK:
        msg = ''
        if handle:
            raw = lib().nicnes_last_error(handle)
            msg = raw.decode() if raw else ''
        cls = DecodeFault if rc == ERR_FAULT else NicnesError
        raise cls('%s failed: %s%s' % (what, _NAMES.get(rc, 'error %d' % rc), (': ' + msg) if msg else ''))
