"""Master/worker transport for the engine, mirroring /root/reference/src/dist.py.

Same keys (dist.py:17-22) and the same client methods (MasterClient.declare_experiment /
declare_task / pop_result / flush_results, WorkerClient.get_experiment / get_current_task /
push_result, dist.py:68-201), with two deliberate differences:

* the wire codec is msgpack with an ndarray extension (dtype string, shape, raw bytes) instead of
  pickle (dist.py:25-30): a message can carry only plain data, decoding never executes anything;
* results are ~100 bytes (fitness pair + noise index) instead of the 11.46 MB noise vector.

`LocalStore` is an in-process, thread-safe subset of the redis commands these clients use, so a
master and its workers can run in one process (tests, single-node) without a redis server. A real
redis server is used when the `redis` package is importable and a redis config dict is given.
"""
import threading
import time
from collections import deque

import msgpack
import numpy as np

from .nes import NESResult, NESTask

EXP_KEY = 'nic:exp'
TASK_ID_KEY = 'nic:task_id'
TASK_DATA_KEY = 'nic:task_data'
TASK_CHANNEL = 'nic:task_channel'
RESULTS_KEY = 'nic:results'
ARCHIVE_KEY = 'nic:archive'
MEMBER_KEY = 'nic:member_counter'       # new: per-task member-id allocator (members are noise indices)

_EXT_NDARRAY, _EXT_TASK, _EXT_RESULT, _EXT_TUPLE = 1, 2, 3, 4


# ---------------------------------------------------------------- codec ---------------------------
def _default(obj):
    if isinstance(obj, NESTask):
        return msgpack.ExtType(_EXT_TASK, serialize(list(obj)))
    if isinstance(obj, NESResult):
        return msgpack.ExtType(_EXT_RESULT, serialize(list(obj)))
    if isinstance(obj, tuple):
        return msgpack.ExtType(_EXT_TUPLE, serialize(list(obj)))
    if isinstance(obj, np.ndarray):
        if obj.dtype.hasobject:
            raise TypeError('object arrays cannot be sent')
        a = np.ascontiguousarray(obj)
        return msgpack.ExtType(_EXT_NDARRAY, msgpack.packb([a.dtype.str, list(a.shape), a.tobytes()]))
    if isinstance(obj, np.generic):
        return obj.item()
    if hasattr(obj, 'detach') and hasattr(obj, 'numpy'):          # torch tensor -> ndarray
        return _default(obj.detach().cpu().numpy())
    raise TypeError('cannot serialize %r' % type(obj))


def _ext_hook(code, data):
    if code == _EXT_NDARRAY:
        dt, shape, raw = msgpack.unpackb(data)
        dt = np.dtype(dt)
        if dt.hasobject:
            raise ValueError('object dtype on the wire')
        return np.frombuffer(raw, dtype=dt).reshape(shape).copy()
    if code == _EXT_TASK:
        return NESTask(*deserialize(data))
    if code == _EXT_RESULT:
        return NESResult(*deserialize(data))
    if code == _EXT_TUPLE:
        return tuple(deserialize(data))
    raise ValueError('unknown extension type %d' % code)


def serialize(x):
    return msgpack.packb(x, default=_default, use_bin_type=True, strict_types=True)


def deserialize(b):
    return msgpack.unpackb(b, ext_hook=_ext_hook, raw=False, strict_map_key=False)


# ---------------------------------------------------------------- in-process store ----------------
class _Pipeline:
    def __init__(self, store):
        self.s, self.ops = store, []

    def __getattr__(self, name):
        fn = getattr(self.s, name)

        def queue(*a, **k):
            self.ops.append((fn, a, k))
            return self
        return queue

    def watch(self, *keys):
        return None

    def multi(self):
        return None

    def execute(self):
        with self.s._cv:
            out = [fn(*a, **k) for fn, a, k in self.ops]
        self.ops = []
        return out

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.ops = []
        return False


class LocalStore:
    """The redis subset dist.py uses: get/set/mget/mset/incrby/rpush/blpop/llen/ltrim/lrange/publish."""

    def __init__(self):
        self._kv, self._lists = {}, {}
        self._cv = threading.Condition(threading.RLock())

    def ping(self):
        return True

    def set(self, k, v):
        with self._cv:
            self._kv[k] = v if isinstance(v, bytes) else str(v).encode()
            return True

    def get(self, k):
        with self._cv:
            return self._kv.get(k)

    def mget(self, keys):
        with self._cv:
            return [self._kv.get(k) for k in keys]

    def mset(self, mapping):
        with self._cv:
            for k, v in mapping.items():
                self.set(k, v)
            return True

    def delete(self, *keys):
        with self._cv:
            n = 0
            for k in keys:
                n += int(self._kv.pop(k, None) is not None) + int(self._lists.pop(k, None) is not None)
            return n

    def incrby(self, k, n=1):
        with self._cv:
            v = int(self._kv.get(k, b'0')) + int(n)
            self._kv[k] = str(v).encode()
            return v

    def rpush(self, k, *vals):
        with self._cv:
            q = self._lists.setdefault(k, deque())
            q.extend(vals)
            self._cv.notify_all()
            return len(q)

    def blpop(self, k, timeout=0):
        deadline = None if not timeout else time.monotonic() + timeout
        with self._cv:
            while not self._lists.get(k):
                left = None if deadline is None else deadline - time.monotonic()
                if left is not None and left <= 0:
                    return None
                self._cv.wait(left)
            return (k, self._lists[k].popleft())

    def llen(self, k):
        with self._cv:
            return len(self._lists.get(k, ()))

    def ltrim(self, k, start, end):
        with self._cv:
            q = list(self._lists.get(k, ()))
            n = len(q)
            s = start if start >= 0 else max(n + start, 0)
            e = end if end >= 0 else n + end
            self._lists[k] = deque(q[s:e + 1])
            return True

    def lrange(self, k, start, end):
        with self._cv:
            q = list(self._lists.get(k, ()))
            e = end if end >= 0 else len(q) + end
            return q[start:e + 1]

    def publish(self, channel, msg):
        return 0

    def pipeline(self):
        return _Pipeline(self)


class _SeqPipeline:
    """pipeline() of stores without transactions: the queued commands run in order on execute()."""

    def __init__(self, store):
        self.s, self.ops = store, []

    def __getattr__(self, name):
        fn = getattr(self.s, name)

        def queue(*a, **k):
            self.ops.append((fn, a, k))
            return self
        return queue

    def watch(self, *keys):
        return None

    def multi(self):
        return None

    def execute(self):
        out = [fn(*a, **k) for fn, a, k in self.ops]
        self.ops = []
        return out

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.ops = []
        return False


class TCPStoreRedis:
    """The same redis subset over torch.distributed.TCPStore, for master and workers in separate
    processes when no redis server exists (this image has none): 'tcp://host:port' in connect().
    mset writes one snapshot key besides the keys, and mget of keys that snapshot holds reads it, so
    a worker never pairs a new task id with old task data. Lists are TCPStore queues."""

    _SNAP = '__nicnes_mset__'

    def __init__(self, host, port, is_master=False, timeout=60.0):
        from datetime import timedelta
        import torch.distributed as dist
        self.host, self.port = host, int(port)
        self.s = dist.TCPStore(host, self.port, is_master=is_master, wait_for_workers=False,
                               timeout=timedelta(seconds=timeout))

    def ping(self):
        return True

    def set(self, k, v):
        self.s.set(k, v if isinstance(v, bytes) else str(v).encode())
        return True

    def get(self, k):
        return self.s.get(k) if self.s.check([k]) else None

    def mset(self, mapping):
        # the snapshot first: a reader that sees a new individual key finds a snapshot holding it
        vals = {k: (v if isinstance(v, bytes) else str(v).encode()) for k, v in mapping.items()}
        self.s.set(self._SNAP, msgpack.packb(vals, use_bin_type=True))
        for k, v in vals.items():
            self.s.set(k, v)
        return True

    def mget(self, keys):
        snap = self.get(self._SNAP)
        if snap is not None:
            d = msgpack.unpackb(snap, raw=False)
            if all(k in d for k in keys):
                return [d[k] for k in keys]
        return [self.get(k) for k in keys]

    def delete(self, *keys):
        return sum(int(self.s.delete_key(k)) for k in keys)

    def incrby(self, k, n=1):
        return int(self.s.add(k, int(n)))

    def rpush(self, k, *vals):
        for v in vals:
            self.s.queue_push(k, v)
        return int(self.s.queue_len(k))

    def blpop(self, k, timeout=0):
        deadline = None if not timeout else time.monotonic() + timeout
        while self.s.queue_len(k) == 0:
            if deadline is not None and time.monotonic() >= deadline:
                return None
            time.sleep(0.002)
        return (k, self.s.queue_pop(k, False))

    def llen(self, k):
        return int(self.s.queue_len(k))

    def ltrim(self, k, start, end):
        if (start, end) != (-1, -1):
            raise NotImplementedError('TCPStoreRedis.ltrim keeps only the newest item (flush_results)')
        while self.s.queue_len(k) > 1:
            self.s.queue_pop(k, False)
        return True

    def publish(self, channel, msg):
        return 0

    def pipeline(self):
        return _SeqPipeline(self)


def connect(cfg):
    """LocalStore / redis-like object -> itself; 'tcp://host:port' -> TCPStoreRedis (client);
    dict -> redis.StrictRedis(**cfg) (needs redis-py)."""
    if cfg is None:
        return LocalStore()
    if hasattr(cfg, 'rpush'):
        return cfg
    if isinstance(cfg, str) and cfg.startswith('tcp://'):
        host, port = cfg[len('tcp://'):].rsplit(':', 1)
        return TCPStoreRedis(host, int(port))
    try:
        import redis
    except ImportError as e:   # pragma: no cover - redis-py is absent from this image
        raise RuntimeError('a redis config was given but the redis package is not installed') from e
    r = redis.StrictRedis(**cfg)
    r.ping()
    return r


def _retry_get(store, key, tries=300, delay=0.05):
    for _ in range(tries):
        if isinstance(key, (list, tuple)):
            vals = store.mget(key)
            if all(v is not None for v in vals):
                return vals
        else:
            v = store.get(key)
            if v is not None:
                return v
        time.sleep(delay)
    raise RuntimeError('{} not set'.format(key))


# ---------------------------------------------------------------- clients -------------------------
class MsgpackCodec:
    """The engine's own wire: msgpack with an ndarray extension (plain data only)."""
    name = 'msgpack'
    serialize = staticmethod(serialize)
    deserialize = staticmethod(deserialize)


class MasterClient:
    """codec: MsgpackCodec (default) or nicnes.refwire.RefPickleCodec (the reference's pickle wire)."""

    def __init__(self, master_redis_cfg=None, codec=None):
        self.task_counter = 0
        self.master_redis = connect(master_redis_cfg)
        self.codec = codec or MsgpackCodec

    def declare_experiment(self, exp):
        self.master_redis.set(EXP_KEY, self.codec.serialize(exp))

    def declare_task(self, task_data):
        task_id = self.task_counter
        self.task_counter += 1
        data = self.codec.serialize(task_data)
        (self.master_redis.pipeline()
         .mset({TASK_ID_KEY: task_id, TASK_DATA_KEY: data, MEMBER_KEY + ':%d' % task_id: 0})
         .publish(TASK_CHANNEL, self.codec.serialize((task_id, data)))
         .execute())
        return task_id

    def pop_result(self, timeout=0):
        item = self.master_redis.blpop(RESULTS_KEY, timeout=timeout)
        if item is None:
            return None, None
        task_id, result = self.codec.deserialize(item[1])
        return task_id, result

    def flush_results(self):
        return max(self.master_redis.pipeline().llen(RESULTS_KEY).ltrim(RESULTS_KEY, -1, -1).execute()[0] - 1, 0)


class WorkerClient:
    """Argument order as in dist.py:162 (relay, master); with one store both are the same."""

    def __init__(self, relay_redis_cfg=None, master_redis_cfg=None, codec=None):
        self.local_redis = connect(relay_redis_cfg)
        self.master_redis = self.local_redis if master_redis_cfg is None else connect(master_redis_cfg)
        self.cached_task_id, self.cached_task_data = None, None
        self.codec = codec or MsgpackCodec

    def get_experiment(self):
        return self.codec.deserialize(_retry_get(self.local_redis, EXP_KEY))

    def get_current_task(self, retry_sleep=0.01):
        """(task_id, task). A task caught half published (its id without its data, or the pair read
        across two declarations) is not taken: the previous task is served meanwhile, or, before the
        first task, the read is retried."""
        while True:
            task_id = int(_retry_get(self.local_redis, TASK_ID_KEY))
            if task_id == self.cached_task_id:
                return self.cached_task_id, self.cached_task_data
            tid, data = self.local_redis.mget([TASK_ID_KEY, TASK_DATA_KEY])
            if tid is not None and data is not None and int(tid) == task_id:
                self.cached_task_id, self.cached_task_data = task_id, self.codec.deserialize(data)
                return self.cached_task_id, self.cached_task_data
            if self.cached_task_id is not None:
                return self.cached_task_id, self.cached_task_data
            time.sleep(retry_sleep)

    def claim_members(self, task_id, count):
        """Atomically reserve member ids [begin, begin+count) of this task (new; members = noise indices)."""
        end = self.master_redis.incrby(MEMBER_KEY + ':%d' % task_id, count)
        return end - count

    def push_result(self, task_id, result):
        self.local_redis.rpush(RESULTS_KEY, self.codec.serialize((task_id, result)))

    def push_results(self, task_id, results):
        if results:
            self.local_redis.rpush(RESULTS_KEY, *[self.codec.serialize((task_id, r)) for r in results])
