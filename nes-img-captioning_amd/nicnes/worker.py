"""python -m nicnes.worker -- the engine's `workers` entry point (src/main.py:75-153, `main.py workers`).

One worker process per GPU, started with the 'spawn' method (a fresh interpreter: nothing GPU-related
is inherited) by a supervisor that never touches a GPU itself and restarts a dead worker as a fresh
process, as the reference's supervisor respawns dead CPU workers (main.py:107-141). Each worker
attaches to the master's store, reads the experiment (EXP_KEY), builds an Engine on its GPU and serves
the current task:

  --wire engine      for the engine's master (EngineMaster.run_dispatched): msgpack wire, member
                     chunks claimed from the per-task counter, results carry noise-table indices;
  --wire reference   for an UNCHANGED reference master (`main.py master`): the reference's pickle
                     wire (nicnes.refwire), results carry the evolve_noise vectors it sums.

Store: --store tcp://host:port (a torch TCPStore the master serves: no redis server in this image),
or the reference's redis pair (--master_host / --master_port / --relay_socket_path, needs redis-py).
`nic:stop_workers` set in the store stops the pool (the reference stops on Ctrl-C / SIGTERM, also
honoured here). Each worker registers its pid under nic:worker_pid:<index>.

    python -m nicnes.worker --num_workers 8 --store tcp://10.0.0.1:29500 --wire engine
"""
import argparse
import importlib
import logging
import os
import signal
import sys
import threading
import time

STOP_KEY = 'nic:stop_workers'
PID_KEY = 'nic:worker_pid:%d'


def parse_args(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument('--algo', default='nic_nes', choices=['nic_nes'])
    ap.add_argument('--master_host', default='localhost')
    ap.add_argument('--master_port', type=int, default=6379)
    ap.add_argument('--relay_socket_path', default=None)
    ap.add_argument('--store', default=None, help='tcp://host:port (TCPStore); default: the redis pair above')
    ap.add_argument('--num_workers', type=int, default=None, help='worker processes (default: visible GPUs)')
    ap.add_argument('--gpus', default=None, help='comma-separated device indices (default 0..num_workers-1)')
    ap.add_argument('--wire', default='engine', choices=['engine', 'reference'])
    ap.add_argument('--chunk', type=int, default=64, help='members evaluated per claim')
    ap.add_argument('--noise_len', type=int, default=1 << 27)
    ap.add_argument('--noise_seed', type=int, default=0)
    ap.add_argument('--table_seed', type=int, default=123)
    ap.add_argument('--df_path', default=None, help="CiderD df file (coco-train-idxs.p / .json / .npz)")
    ap.add_argument('--vocab_size', type=int, default=9487)
    ap.add_argument('--eval_prob', type=float, default=None, help='reference wire: default config.eval_prob')
    ap.add_argument('--engine_factory', default='nicnes.worker:default_engine')
    ap.add_argument('--check_interval', type=float, default=60.0)
    ap.add_argument('--max_restarts', type=int, default=20, help='restarts allowed within --restart_window seconds')
    ap.add_argument('--restart_window', type=float, default=3600.0)
    ap.add_argument('--max_tasks', type=int, default=None)
    ap.add_argument('--data_root', default='.', help="directory the experiment's caption_options paths are "
                                                     "relative to (the reference runs from src/)")
    return ap.parse_args(argv)


def store_cfg(args):
    if args.store:
        return args.store
    master = {'host': args.master_host, 'port': args.master_port}
    relay = {'unix_socket_path': args.relay_socket_path} if args.relay_socket_path else master
    return relay, master


def default_engine(spec, args, device):
    """An Engine on `device` for the experiment: the shared table, the df table of --df_path."""
    import numpy as np
    import nicnes
    import nicnes.synthetic as S
    from nicnes import data
    from nicnes.nes import EngineWorker
    eng = nicnes.Engine(device=device, **spec.engine_kwargs(max_members=args.chunk, noise_len=args.noise_len,
                                                             noise_seed=args.noise_seed))
    eng.set_noise_table(S.noise_table(args.noise_len, args.table_seed))
    if args.df_path:
        df, ref_len_raw = data.load_df_table(args.df_path)
    else:
        logging.warning('no --df_path: CIDEr-D runs with an empty document-frequency table')
        df, ref_len_raw = {}, 1.0
    keys, vals = nicnes.df_table_arrays(df)
    eng.set_df_table(keys, vals, np.log(float(ref_len_raw)))
    return eng, EngineWorker(eng, spec, worker_id=os.getpid())


def _factory(path):
    mod, fn = path.split(':')
    return getattr(importlib.import_module(mod), fn)


def worker_main(index, device, args, shared_device=False):
    """One worker process: engine on `device`, then the serve loop until the stop key is set.
    shared_device: another worker of this pool runs on the same GPU. The coop decode then stays off: its
    workgroups wait for each other and assume the whole device, which a second process's kernels break
    (a stalled hand-off is a contained fault, but every later evaluate of the worker then fails)."""
    logging.basicConfig(format='[%(asctime)s pid=%(process)d] %(message)s', level=logging.INFO)
    from nicnes import config as C
    from nicnes import transport as T
    from nicnes import master as M
    from nicnes import refwire as W
    codec = W.RefPickleCodec if args.wire == 'reference' else T.MsgpackCodec
    cfg = store_cfg(args)
    client = T.WorkerClient(*cfg, codec=codec) if isinstance(cfg, tuple) else T.WorkerClient(cfg, codec=codec)
    client.local_redis.set(PID_KEY % index, str(os.getpid()))
    exp = client.get_experiment()
    spec = C.ExperimentSpec(exp, vocab_size=args.vocab_size)
    engine, worker = _factory(args.engine_factory)(spec, args, device)
    if shared_device and hasattr(engine, 'set_decode_coop'):
        engine.set_decode_coop(0)
    stop = threading.Event()

    def watch():
        while not stop.is_set():
            if client.local_redis.get(STOP_KEY) is not None:
                stop.set()
            time.sleep(0.05)
    threading.Thread(target=watch, daemon=True).start()
    logging.info('worker %d on device %s serving the %s wire', index, device, args.wire)
    if args.wire == 'reference':
        eval_prob = args.eval_prob if args.eval_prob is not None else float(spec.config.eval_prob or 0.0)
        own = None
        if not spec.single_batch:
            # single_batch: false -- each member on a batch of this worker's own loader (nic_nes_worker.py:121-128),
            # shuffled by its own seed as each reference worker process shuffles independently
            from nicnes import data as Dt
            try:
                own = W.OwnBatches(lambda bs: Dt.loader_from_caption_options(spec.exp, bs, seed=os.getpid(),
                                                                             root=args.data_root),
                                   spec.batch_size)
            except FileNotFoundError as e:
                logging.warning('no caption data for an own loader (%s)', e)
        W.run_reference_worker(client, worker, chunk=args.chunk, eval_prob=eval_prob, stop=stop,
                               max_tasks=args.max_tasks, own_batches=own)
    else:
        M.run_worker(client, worker, chunk=args.chunk, stop=stop, max_tasks=args.max_tasks)
    stop.set()
    if hasattr(engine, 'close'):
        engine.close()


def _visible_gpus():
    try:
        import torch
        return torch.cuda.device_count()          # counts devices without initialising HIP
    except Exception:
        return 0


class RestartBudget:
    """At most `max_restarts` restarts within any `window` seconds (a rate, not a lifetime total: a
    long run that loses a worker now and then, e.g. to the parameter-file race of
    nic_nes_worker.py:71-84, keeps its pool)."""

    def __init__(self, max_restarts, window):
        self.max, self.window, self.times = int(max_restarts), float(window), []

    def allow(self, now):
        self.times = [t for t in self.times if now - t < self.window]
        if len(self.times) >= self.max:
            return False
        self.times.append(now)
        return True


def supervise(args):
    """Start one worker per GPU, restart dead ones as fresh processes, stop on SIGINT / SIGTERM or
    the store's stop key. Returns the number of restarts."""
    import multiprocessing as mp
    from nicnes import transport as T
    logging.basicConfig(format='[%(asctime)s pid=%(process)d] %(message)s', level=logging.INFO)
    n = args.num_workers or max(_visible_gpus(), 1)
    devices = [int(g) for g in args.gpus.split(',')] if args.gpus else list(range(n))
    if len(devices) < n:
        raise SystemExit('--gpus names %d devices for %d workers' % (len(devices), n))
    ctx = mp.get_context('spawn')
    cfg = store_cfg(args)
    store = T.connect(cfg[0] if isinstance(cfg, tuple) else cfg)

    def start(i):
        shared = devices[:n].count(devices[i]) > 1
        p = ctx.Process(target=worker_main, args=(i, devices[i], args, shared), name='nicnes-worker-%d' % i)
        p.start()
        return p

    procs = {i: start(i) for i in range(n)}
    stopping = threading.Event()
    for sig in (signal.SIGINT, signal.SIGTERM):
        signal.signal(sig, lambda *_: stopping.set())
    restarts = 0
    budget = RestartBudget(args.max_restarts, getattr(args, 'restart_window', 3600.0))
    try:
        while not stopping.is_set():
            if store.get(STOP_KEY) is not None:
                break
            for i, p in list(procs.items()):
                if not p.is_alive():
                    if not budget.allow(time.monotonic()):
                        logging.warning('worker %d died (exit %s); restart budget spent', i, p.exitcode)
                        stopping.set()
                        break
                    logging.warning('worker %d died (exit %s): starting a fresh process', i, p.exitcode)
                    procs[i] = start(i)
                    restarts += 1
            stopping.wait(args.check_interval)
    finally:
        deadline = time.time() + 30
        for p in procs.values():
            p.join(max(deadline - time.time(), 0.1))
        for p in procs.values():
            if p.is_alive():
                p.terminate()
                p.join(5)
            if p.is_alive():
                p.kill()
    logging.info('worker pool stopped after %d restart(s)', restarts)
    return restarts


def main(argv=None):
    args = parse_args(argv)
    supervise(args)
    return 0


if __name__ == '__main__':
    sys.exit(main())
