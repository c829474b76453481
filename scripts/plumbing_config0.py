"""BASELINE.json configs[0] -- 'mnist_nes.json, pop=16, 1 CPU worker via src/scripts/local_run_exp.sh
(plumbing, no GPU)' -- on the build's own harness.

The reference cannot run here (no redis-server, no torchvision / MNIST download, its from_infos log
is absent). What this exercises instead is the same plumbing: a master process
and ONE worker process (`python -m nicnes.worker --num_workers 1`, as local_run_exp.sh starts
`main.py master` + `main.py workers`) exchanging NESTask / NESResult over a store, with
mnist_nes.json's config values (noise_stdev 0.02, batch_size 64 -> here the tiny workload's images,
l2coeff 1e-3, Adam stepsize 0.01, single_batch false, stdev_divisor 2 / bs_multiplier 2) at pop = 16.
The MNIST CNN, vbn and SM-G-SUM are outside the engine's path: the net is the fc_caption captioner of
the tiny oracle workload (CPU, no GPU), evaluated by the oracle engine in the worker.
Prints one JSON record (committed as profiles/r02_config0_plumbing.json)."""
import json
import os
import signal
import socket
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, 'nes-img-captioning_amd'))

import numpy as np  # noqa: E402

from nicnes import config as C, master as M, transport as T  # noqa: E402
from nicnes.worker import STOP_KEY  # noqa: E402
from tests.cpu_engine import OracleEngine, tiny_workload  # noqa: E402

MNIST_NES = {   # /root/reference/experiments/mnist_nes.json, config / optimizer values
    'eval_prob': 0.1, 'noise_stdev': 0.02, 'snapshot_freq': 5, 'batch_size': 64, 'patience': 2, 'stdev_divisor': 2,
    'bs_multiplier': 2, 'stepsize_divisor': 1, 'ref_batch_size': 16, 'l2coeff': 0.001, 'single_batch': False}


def main(iterations=3, pop=16):
    dims, theta, fc, gts, df, n, table = tiny_workload(B=8)
    cfg = dict(MNIST_NES, batch_size=4, snapshot_freq=0)          # the tiny workload's images per batch
    exp = {'algorithm': 'nic_nes', 'dataset': 'mscoco', 'nb_offspring': pop, 'batches_per_iteration': 2,
           'config': cfg, 'policy_options': {'net': 'fc_caption', 'fitness': 'greedy', 'model_options': {}},
           'optimizer_options': {'type': 'adam', 'args': {'stepsize': 0.01}}}
    spec = C.ExperimentSpec(exp, vocab_size=63)
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    store = T.TCPStoreRedis('127.0.0.1', port, is_master=True)
    env = dict(os.environ, PYTHONPATH=os.pathsep.join([REPO, os.path.join(REPO, 'nes-img-captioning_amd')]))
    cmd = [sys.executable, '-m', 'nicnes.worker', '--store', 'tcp://127.0.0.1:%d' % port, '--num_workers', '1',
           '--wire', 'engine', '--engine_factory', 'tests.worker_factory:oracle_engine', '--vocab_size', '63',
           '--chunk', '4', '--check_interval', '0.5', '--noise_seed', '0']
    t0 = time.time()
    pool = subprocess.Popen(cmd, env=env, cwd=REPO, start_new_session=True, stdout=subprocess.DEVNULL,
                            stderr=subprocess.DEVNULL)
    try:
        master = M.EngineMaster(spec, OracleEngine(dims, theta, fc, gts, df, n, table), log_dir='/tmp/nicnes_config0')
        batches = [[{'fc_feats': fc[4 * g: 4 * g + 4], 'gts': gts[4 * g: 4 * g + 4]} for g in range(2)]] * iterations
        master.run_dispatched(T.MasterClient(store), batches, max_iterations=iterations, result_timeout=300)
        store.set(STOP_KEY, b'1')
        rc = pool.wait(timeout=120)
    finally:
        if pool.poll() is None:
            os.killpg(pool.pid, signal.SIGKILL)
    rec = {'config': 'BASELINE.json configs[0]: mnist_nes.json, pop=16, 1 CPU worker (plumbing, no GPU)',
           'reference': 'not runnable here (redis-server, torchvision/MNIST download, from_infos log absent)',
           'harness': 'master process + `python -m nicnes.worker --num_workers 1` over a TCPStore, oracle engine (CPU)',
           'net': 'fc_caption tiny (V=63, E=R=32, F=64): the MNIST CNN, vbn and SM-G-SUM are outside the engine',
           'population': pop, 'iterations': master.sched.iteration, 'worker_exit_code': rc,
           'score_mean': [round(r['score_mean'], 6) for r in master.stats],
           'update_ratio': [round(r['update_ratio'], 8) for r in master.stats],
           'wall_s': round(time.time() - t0, 2)}
    print(json.dumps(rec))
    return rec


if __name__ == '__main__':
    main()
