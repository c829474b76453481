"""The reference's own wire, so engine workers can serve an UNCHANGED reference master.

The reference pickles everything it puts on redis (src/dist.py:25-30, protocol -1): the master's
NESTask (src/algorithm/nic_nes/nic_nes_master.py:27-28, declared at :79-85) and each worker's
(task_id, NESResult) (:30-31, pushed at src/dist.py:199-201, built at
src/algorithm/nic_nes/nic_nes_worker.py:156-161). Its master then reads
result.fitness / result.evolve_noise / result.eval_score (nic_nes_master.py:92-123).

  dumps(obj)   pickle bytes whose wire-type globals are the reference's own classes
               (algorithm.nic_nes.nic_nes_master.NESTask / NESResult), written without importing
               the reference: RefNESTask / RefNESResult carry the reference's module path, and the
               pickler emits that path for them. Everything else (numpy arrays, dicts, floats) is
               pickled as the reference pickles it, byte for byte (tests/test_worker_entry.py,
               test_engine_results_are_the_reference_bytes, checks the bytes against the reference's own
               dist.serialize output, tests/golden/wire_reference.npz).
  loads(b)     a restricted unpickler: the reference wire types map to RefNESTask / RefNESResult, and
               only numpy array / scalar reconstruction and a few plain containers are admitted; any
               other global (os.system, builtins.eval, ...) is refused, so decoding never runs code.
  RefPickleCodec   the serialize / deserialize pair for nicnes.transport clients (codec=...).
  run_reference_worker
               NESWorker.run_worker (nic_nes_worker.py:41-90) on the engine: members in chunks, each
               result in the reference format with its evolve_noise = fp32(sigma * z) materialised
               from the shared table (nicnes_noise_vectors). Each claimed slot of a chunk is, with
               probability eval_prob, an eval result instead of a member, as each reference worker
               iteration is (nic_nes_worker.py:65): the greedy CIDEr-D fitness of the unperturbed theta
               on the task batch stands in for the COCO validation eval, which needs java and the val
               set (out of scope).
               With single_batch: false (mscoco_nes.json's setting) each member is scored on a batch
               drawn from the worker's own loader (OwnBatches), as each reference fitness call draws one
               (nic_nes_worker.py:121-128); the SM-G-SUM sensitivity of a task is computed on the first
               of them (the reference computes it once per task, on its first fitness call's batch:
               nic_nes_worker.py:139-140, safe_mutations.py:34-40). Without a loader (no caption data
               on the worker) members fall back to the published batch, with a warning.
"""
import logging
import io
import os
import pickle
import random
import time
from collections import namedtuple

import numpy as np

from .nes import NESTask, ParameterFileError

REF_MODULE = 'algorithm.nic_nes.nic_nes_master'

ref_task_fields = ['current', 'batch_data', 'noise_stdev', 'log_dir', 'ref_batch', 'batch_size']
RefNESTask = namedtuple('NESTask', field_names=ref_task_fields, defaults=(None,) * len(ref_task_fields))
RefNESTask._ref_global = (REF_MODULE, 'NESTask')

ref_result_fields = ['worker_id', 'eval_score', 'evolve_noise', 'fitness', 'mem_usage']
RefNESResult = namedtuple('NESResult', field_names=ref_result_fields, defaults=(None,) * len(ref_result_fields))
RefNESResult._ref_global = (REF_MODULE, 'NESResult')


class _RefPickler(pickle._Pickler):
    """The standard (pure-Python) pickler, except that classes marked with _ref_global are written
    as that global -- the way the reference's pickler writes its own namedtuple classes."""

    def save_global(self, obj, name=None):
        ref = getattr(obj, '_ref_global', None) if isinstance(obj, type) else None
        if ref is None:
            return super().save_global(obj, name)
        module, qualname = ref
        if self.proto >= 4:
            self.save(module)
            self.save(qualname)
            self.write(pickle.STACK_GLOBAL)
        else:
            self.write(pickle.GLOBAL + bytes(module, 'utf-8') + b'\n' + bytes(qualname, 'utf-8') + b'\n')
        self.memoize(obj)


def dumps(obj, protocol=pickle.HIGHEST_PROTOCOL):
    """dist.serialize (pickle.dumps(x, protocol=-1)) with the reference's wire types."""
    f = io.BytesIO()
    _RefPickler(f, protocol).dump(obj)
    return f.getvalue()


def _numpy_globals():
    """numpy's pickle reconstructors under both of their module paths (numpy 1.x writes numpy.core,
    numpy 2.x numpy._core)."""
    try:
        from numpy._core import multiarray as ma, numeric as nu
    except ImportError:                   # numpy 1.x
        from numpy.core import multiarray as ma, numeric as nu
    out = {('numpy', 'ndarray'): np.ndarray, ('numpy', 'dtype'): np.dtype}
    for root in ('numpy.core', 'numpy._core'):
        out[(root + '.multiarray', '_reconstruct')] = ma._reconstruct
        out[(root + '.multiarray', 'scalar')] = ma.scalar
        out[(root + '.numeric', '_frombuffer')] = nu._frombuffer
    return out


_ALLOWED = None


class _RefUnpickler(pickle.Unpickler):
    def find_class(self, module, name):
        global _ALLOWED
        if _ALLOWED is None:
            import collections
            _ALLOWED = dict(_numpy_globals())
            _ALLOWED.update({(REF_MODULE, 'NESTask'): RefNESTask, (REF_MODULE, 'NESResult'): RefNESResult,
                             ('collections', 'OrderedDict'): collections.OrderedDict,
                             ('builtins', 'set'): set, ('builtins', 'frozenset'): frozenset,
                             ('builtins', 'complex'): complex})
        try:
            return _ALLOWED[(module, name)]
        except KeyError:
            raise pickle.UnpicklingError('global %s.%s is not allowed on the wire' % (module, name)) from None


def loads(b):
    return _RefUnpickler(io.BytesIO(b)).load()


class RefPickleCodec:
    """serialize / deserialize of nicnes.transport clients for the reference's redis protocol."""
    name = 'reference-pickle'

    @staticmethod
    def serialize(x):
        return dumps(x)

    @staticmethod
    def deserialize(b):
        return loads(b)


def to_engine_task(ref_task, task_id):
    """A reference NESTask -> the engine's (the task id is the noise-rule iteration: the reference
    task carries no iteration counter)."""
    return NESTask(current=ref_task.current, batch_data=ref_task.batch_data, noise_stdev=ref_task.noise_stdev,
                   log_dir=ref_task.log_dir, ref_batch=ref_task.ref_batch, batch_size=ref_task.batch_size,
                   iteration=int(task_id))


def _rss():
    try:
        import psutil
        return int(psutil.Process(os.getpid()).memory_info().rss)
    except Exception:          # pragma: no cover - psutil is present in this image
        return 0


class OwnBatches:
    """A reference worker's own training loader (single_batch: false, nic_nes_worker.py:121-128): draw(bs)
    returns its next training batch. When the task's batch_size differs from the loader's, the loader is
    made anew at that size, as Experiment.increase_loader_batch_size re-runs init_loaders (a new DataLoader:
    algorithm/tools/experiment.py:64-65, captioning/experiment.py:33-44). make_loader(batch_size) builds
    one (e.g. nicnes.data.loader_from_caption_options)."""

    def __init__(self, make_loader, batch_size):
        self.make = make_loader
        self.loader = make_loader(int(batch_size))

    def draw(self, batch_size=None):
        if batch_size is not None and int(batch_size) != self.loader.batch_size:
            self.loader = self.make(int(batch_size))
        return self.loader.get_batch('train')


def reference_results(worker, task_id, task, member_begin, count, batches=None):
    """The engine's evaluation of members [member_begin, +count) as reference NESResults
    (fitness = (f+, f-), evolve_noise = the member's delta). batches: one batch per member (own loader)."""
    kw = {} if batches is None else {'batches': batches}
    res = worker.fitness_batch(task_id, task, member_begin, count, **kw)
    it = int(task.iteration)
    deltas = worker.e.noise_vectors(it, member_begin, count, float(task.noise_stdev)).cpu().numpy()
    mem = _rss()
    return [RefNESResult(worker_id=worker.worker_id, evolve_noise=np.ascontiguousarray(deltas[k]),
                         fitness=np.asarray(r.fitness, np.float64), mem_usage=mem) for k, r in enumerate(res)]


# what the reference worker survives (nic_nes_worker.py:71-84: the master deletes and rewrites the current
# parameter file between iterations, so a late reader can find it missing or half written). Only the
# parameter-file race: an engine error (NicnesError, e.g. a contained decode fault) or a HIP error ends the
# worker process with a nonzero status, and the supervisor (nicnes.worker) starts a fresh one.
TRANSIENT_ERRORS = (FileNotFoundError, ParameterFileError)


def chunk_evals(rs, chunk, eval_prob):
    """How many of a chunk's `chunk` slots are eval runs: one eval_prob coin per slot, as one per
    reference worker iteration (nic_nes_worker.py:65), so the master sees eval results at the
    reference's rate per result whatever the chunk size."""
    if not eval_prob:
        return 0
    return sum(1 for _ in range(chunk) if rs.random() < eval_prob)


def run_reference_worker(client, worker, chunk=16, eval_prob=0.0, max_tasks=None, stop=None, seed=None,
                         idle_sleep=0.005, max_results=None, retry_sleep=0.05, own_batches=None):
    """NESWorker.run_worker (nic_nes_worker.py:41-90) against a reference master: `client` is a
    nicnes.transport.WorkerClient built with codec=RefPickleCodec. Each pass takes `chunk` slots:
    chunk_evals of them are eval results (one rollout of the unperturbed theta, pushed once per eval
    slot), the rest are members claimed from a per-task counter in the same store (the reference's
    workers draw their noise independently; the engine needs distinct noise indices). Results of a
    task keep flowing until the master declares the next one, as reference workers do (surplus results
    are dropped by the master, nic_nes_master.py:108-116). A missing or half-written parameter file is
    logged and the task re-read, as nic_nes_worker.py:71-84 does. With single_batch: false and own_batches (an
    OwnBatches), each member slot draws its batch from it at the task's batch_size. Returns the number of
    tasks seen."""
    rs = random.Random(seed)
    log = logging.getLogger(__name__)
    spec = getattr(worker, 'spec', None)
    own = own_batches if (spec is not None and not getattr(spec, 'single_batch', True)) else None
    if spec is not None and not getattr(spec, 'single_batch', True) and own is None:
        log.warning('single_batch is false but this worker has no loader of its own (caption_options data): every '
                    'member is scored on the published batch, not on one of its own (nic_nes_worker.py:121-128)')
    seen, pushed = set(), 0
    while not (stop is not None and stop.is_set()):
        task_id, ref_task = client.get_current_task()
        if max_tasks is not None and task_id not in seen and len(seen) >= max_tasks:
            return len(seen)
        seen.add(task_id)
        task = to_engine_task(ref_task, task_id)
        n_eval = chunk_evals(rs, chunk, eval_prob)
        try:
            if n_eval:
                worker._prepare(task_id, task)
                score = worker.policy.rollout(None, task.batch_data, None)
                ev = RefNESResult(worker_id=worker.worker_id, eval_score=score, mem_usage=_rss())
                client.push_results(task_id, [ev] * n_eval)
                pushed += n_eval
            if chunk > n_eval:
                n = chunk - n_eval
                batches = [own.draw(task.batch_size) for _ in range(n)] if own is not None else None
                begin = client.claim_members(task_id, n)
                client.push_results(task_id, reference_results(worker, task_id, task, begin, n, batches=batches))
                pushed += chunk - n_eval
        except TRANSIENT_ERRORS as e:
            log.error('task %s: %s (re-reading the task)', task_id, e)
            time.sleep(retry_sleep)
            continue
        if max_results is not None and pushed >= max_results:
            return len(seen)
        time.sleep(idle_sleep)
    return len(seen)
