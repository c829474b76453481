"""CPU tests of the reference-facing layer: experiment JSON surface, wire codec and in-process
store, theta <-> state_dict, optimizer files, and the master/worker loops (dispatched over the
transport vs the sharded local loop) on the oracle-backed CPU engine."""
import threading

import numpy as np
import pytest
import torch

from nicnes import config as C
from nicnes import master as M
from nicnes import nes as N
from nicnes import transport as T
from oracle import cider_ref as CR
from oracle import oracle as O
from tests.cpu_engine import OracleEngine, tiny_workload

# the keys of /root/reference/experiments/mscoco_nes.json (values as in that file)
MSCOCO_NES = {
    'algorithm': 'nic_nes',
    'config': {'eval_prob': 0.003, 'noise_stdev': 0.01, 'snapshot_freq': 5, 'batch_size': 64, 'val_batch_size': 256,
               'num_val_items': 5000, 'patience': 0, 'schedule_start': 1000, 'schedule_limit': 1000,
               'stdev_divisor': 1, 'bs_multiplier': 1, 'stepsize_divisor': 1, 'ref_batch_size': 0, 'l2coeff': 1e-7,
               'single_batch': False},
    'policy_options': {'net': 'fc_caption', 'fitness': 'greedy', 'vbn': False,
                       'model_options': {'safe_mutations': '', 'safe_mutation_vector': '',
                                         'safe_mutation_underflow': 0.1, 'vbn_e': False, 'vbn_affine': False,
                                         'layer_n': False, 'layer_n_affine': False, 'input_encoding_size': 128,
                                         'rnn_size': 128, 'fc_feat_size': 2048}},
    'optimizer_options': {'type': 'adam', 'args': {'stepsize': 0.001}},
    'dataset': 'mscoco', 'nb_offspring': 2000, 'num_elites': 1, 'from_single': './pretrained/bu_xent_09.pth',
    '_from_infos': 'logs/x/snapshot/z_info_e1_i716-885.json',
}


def _exp(**over):
    import copy
    e = copy.deepcopy(MSCOCO_NES)
    for k, v in over.items():
        if isinstance(v, dict) and isinstance(e.get(k), dict):
            e[k].update(v)
        else:
            e[k] = v
    return e


# ------------------------------------------------------------------ config -------------------------
def test_spec_reads_mscoco_nes():
    s = C.ExperimentSpec(MSCOCO_NES)
    assert s.sigma == 0.01 and s.batch_size == 64 and s.l2coeff == 1e-7 and s.nb_offspring == 2000
    assert s.optimizer_type == 'adam' and s.optimizer_args == {'stepsize': 0.001}
    assert 'from_infos' not in s.exp and '_from_infos' not in s.exp
    kw = s.engine_kwargs(max_members=512)
    assert (kw['vocab_size'], kw['input_encoding_size'], kw['rnn_size'], kw['fc_feat_size'], kw['seq_length']) == \
        (9487, 128, 128, 2048, 16)


@pytest.mark.parametrize('over', [
    {'policy_options': {'net': 'fc_caption', 'fitness': 'beam'}},
    {'policy_options': {'net': 'att_caption'}},
    {'policy_options': {'net': 'fc_caption', 'vbn': True}},
    {'policy_options': {'net': 'fc_caption', 'model_options': {'safe_mutations': 'SM-G-ABS'}}},
    {'policy_options': {'net': 'fc_caption', 'model_options': {'safe_mutations': 'SM-OTHER'}}},
    {'optimizer_options': {'type': 'rmsprop', 'args': {}}},
    {'algorithm': 'nic_es'},
])
def test_spec_rejects_unsupported(over):
    with pytest.raises(C.NotSupported):
        C.ExperimentSpec(_exp(**over))


@pytest.mark.parametrize('fitness', ['greedy', 'greedy_logprob', 'greedy_expprob', 'greedy_linprob',
                                     'greedy_avgprob', 'sample', 'self_critical', 'sc_loss', None])
def test_spec_accepts_fitness_modes(fitness):
    """Every Fitness value (src/captioning/policies.py:22-35); None -> Fitness.DEFAULT 'greedy'."""
    s = C.ExperimentSpec(_exp(policy_options={'net': 'fc_caption', 'fitness': fitness}))
    assert s.fitness == (fitness or 'greedy')


# ------------------------------------------------------------------ codec / store ------------------
def test_codec_roundtrip_task_and_result():
    gts = [np.arange(32, dtype=np.int64).reshape(2, 16), np.zeros((5, 16), np.int64)]
    task = N.NESTask(current='/tmp/x.pth', batch_data={'fc_feats': np.ones((10, 8), np.float32), 'gts': gts},
                     noise_stdev=0.01, batch_size=2, iteration=3)
    t2 = T.deserialize(T.serialize((7, task)))
    assert t2[0] == 7 and isinstance(t2[1], N.NESTask)
    b = t2[1].batch_data
    assert b['fc_feats'].dtype == np.float32 and np.array_equal(b['fc_feats'], task.batch_data['fc_feats'])
    assert all(np.array_equal(x, y) and x.dtype == y.dtype for x, y in zip(b['gts'], gts))
    assert t2[1].noise_stdev == 0.01 and t2[1].iteration == 3 and t2[1].ref_batch is None
    r = N.NESResult(worker_id=5, fitness=np.array([1.5, 2.5]), noise_idx=np.int64(640), member=3)
    r2 = T.deserialize(T.serialize(r))
    assert isinstance(r2, N.NESResult) and r2.noise_idx == 640 and np.array_equal(r2.fitness, r.fitness)
    assert r2.evolve_noise is None


def test_codec_refuses_objects():
    with pytest.raises(TypeError):
        T.serialize(np.array([object()], dtype=object))
    with pytest.raises(TypeError):
        T.serialize({'f': lambda: 0})
    import msgpack
    with pytest.raises(ValueError):
        T.deserialize(msgpack.packb(msgpack.ExtType(99, b'')))


def test_local_store_semantics():
    s = T.LocalStore()
    assert s.blpop('q', timeout=0.01) is None
    s.rpush('q', b'a', b'b', b'c')
    assert s.llen('q') == 3 and s.blpop('q')[1] == b'a'
    # MasterClient.flush_results keeps the last element and reports how many were dropped
    mc = T.MasterClient(s)
    s.rpush(T.RESULTS_KEY, b'1', b'2', b'3')
    assert mc.flush_results() == 2 and s.llen(T.RESULTS_KEY) == 1
    assert s.incrby('c', 4) == 4 and s.incrby('c', 4) == 8
    out = s.pipeline().mset({'x': 1}).get('x').execute()
    assert out[1] == b'1'


def test_clients_task_cache_and_member_claims():
    s = T.LocalStore()
    mc, wc = T.MasterClient(s), T.WorkerClient(s)
    mc.declare_experiment({'a': 1})
    assert wc.get_experiment() == {'a': 1}
    t0 = mc.declare_task(N.NESTask(noise_stdev=0.5))
    assert wc.get_current_task()[0] == t0 == 0
    assert wc.claim_members(t0, 8) == 0 and wc.claim_members(t0, 8) == 8
    t1 = mc.declare_task(N.NESTask(noise_stdev=0.25))
    tid, task = wc.get_current_task()
    assert tid == t1 == 1 and task.noise_stdev == 0.25
    assert wc.claim_members(t1, 4) == 0
    wc.push_result(t1, N.NESResult(fitness=np.zeros(2), member=0))
    tid, res = mc.pop_result(timeout=1)
    assert tid == 1 and res.member == 0


# ------------------------------------------------------------------ policy / optimizer files -------
@pytest.fixture(scope='module')
def workload():
    return tiny_workload(B=4)


def _engine(workload):
    dims, theta, fc, gts, df, n, table = workload
    return OracleEngine(dims, theta, fc, gts, df, np.log(float(n)), table)


def test_state_dict_roundtrip_and_set_model(workload, tmp_path):
    e = _engine(workload)
    pol = N.EnginePolicy(e)
    sd = pol.state_dict()
    assert list(sd) == N.PARAM_NAMES
    assert all(tuple(sd[k].shape) == shp for k, shp in N.param_shapes(e).items())
    vec = N.vector_from_state_dict(sd, N.param_shapes(e))
    assert np.array_equal(vec.numpy(), workload[1])
    p = str(tmp_path / 'cur.pth')
    sd64 = {k: v.double() * 2 for k, v in sd.items()}
    torch.save(sd64, p)
    pol.set_model(p)
    assert np.array_equal(e.theta32, (workload[1].astype(np.float64) * 2).astype(np.float32))
    bad = dict(sd)
    bad.pop('core.h2h.bias')
    with pytest.raises(KeyError):
        pol.set_model(bad)
    bad = dict(sd, **{'logit.bias': torch.zeros(3)})
    with pytest.raises(ValueError):
        pol.set_model(bad)


def test_unique_batch():
    fc = np.arange(40, dtype=np.float32).reshape(10, 4)
    gts = [np.zeros((5, 16)), np.zeros((5, 16))]
    u, g = N.unique_batch({'fc_feats': fc, 'gts': gts})
    assert u.shape == (2, 4) and np.array_equal(u, fc[[0, 5]])
    with pytest.raises(ValueError):
        N.unique_batch({'fc_feats': fc[:3], 'gts': gts})


def test_optimizer_file_reads_reference_layout(tmp_path):
    """The reference saves m, v as numpy arrays (optimizers.py:85-95); they load under weights_only."""
    p = str(tmp_path / 'optimizer.tar')
    m, v = np.linspace(0, 1, 7), np.linspace(1, 2, 7)
    torch.save({'dim': 7, 't': 3, 'stepsize': 0.5, 'beta1': 0.8, 'beta2': 0.9, 'epsilon': 1e-6, 'm': m, 'v': v}, p)
    st = N._load_state(p)
    assert st['t'] == 3 and np.array_equal(st['m'], m) and np.array_equal(st['v'], v)


# ------------------------------------------------------------------ master loops ---------------------
def _spec(P, opt='adam', fitness='greedy'):
    return C.ExperimentSpec(_exp(nb_offspring=P, config={'noise_stdev': 0.05, 'batch_size': 4, 'l2coeff': 1e-3,
                                                         'snapshot_freq': 1},
                                 policy_options={'net': 'fc_caption', 'fitness': fitness},
                                 optimizer_options={'type': opt, 'args': {'stepsize': 0.01}}), vocab_size=63)


@pytest.mark.parametrize('opt', ['adam', 'sgd'])
def test_dispatched_loop_matches_local_loop(workload, tmp_path, opt):
    dims, theta, fc, gts, df, n, table = workload
    P, iters = 6, 2
    batch = {'fc_feats': fc, 'gts': gts}

    local = M.EngineMaster(_spec(P, opt), _engine(workload), log_dir=str(tmp_path / 'a'))
    local.run([batch], max_iterations=iters)

    e_master, e_worker = _engine(workload), _engine(workload)
    master = M.EngineMaster(_spec(P, opt), e_master, log_dir=str(tmp_path / 'b'))
    store = T.LocalStore()
    worker = N.EngineWorker(e_worker, _spec(P, opt), worker_id=1)
    th = threading.Thread(target=M.run_worker, args=(T.WorkerClient(store), worker),
                          kwargs=dict(chunk=4, max_tasks=iters), daemon=True)
    th.start()
    master.run_dispatched(T.MasterClient(store), [batch] * iters, max_iterations=iters, result_timeout=120)
    th.join(timeout=120)
    assert not th.is_alive()

    a64, a32 = local.e.theta()
    b64, b32 = master.e.theta()
    assert np.array_equal(a64.numpy(), b64.numpy())
    assert [r['score_mean'] for r in local.stats] == [r['score_mean'] for r in master.stats]
    assert local.opt.t == iters == master.opt.t


def test_worker_fitness_follows_spec_criterion(workload):
    """EngineWorker built from a greedy_linprob spec scores members with the criterion
    (CaptPolicy.rollout, policies.py:119-123), not with 100 * CIDEr."""
    dims, theta, fc, gts, df, n, table = workload
    batch = {'fc_feats': fc, 'gts': gts}
    task = N.NESTask(current=None, batch_data=batch, noise_stdev=0.05, batch_size=4, iteration=1)
    e = _engine(workload)
    res = N.EngineWorker(e, _spec(2, 'adam', 'greedy_linprob'), worker_id=1).fitness_batch(0, task, 0, 2)
    assert e.fitness_mode == 3
    idx = O.noise_index(0, 1, 1, table.size, dims.D)
    seq, lp, _ = O.decode(dims, O.perturb(theta, table, idx, 0.05, -1), fc)
    _, scores = CR.rollout_fitness(e.scorer, seq, gts)
    assert res[1].fitness[1] == CR.criterion_fitness('greedy_linprob', lp, seq, scores)


def test_snapshot_roundtrip(workload, tmp_path):
    P = 4
    m1 = M.EngineMaster(_spec(P), _engine(workload), log_dir=str(tmp_path))
    m1.run([{'fc_feats': workload[2], 'gts': workload[3]}], max_iterations=1)
    import glob
    info = glob.glob(str(tmp_path / 'snapshot' / 'z_info_e*_i1-*.json'))
    assert len(info) == 1
    sd = torch.load(m1.current_model_path(), weights_only=True)
    assert sd['logit.weight'].dtype == torch.float64          # fp64 master after the first update
    st = N._load_state(str(tmp_path / 'snapshot' / 'optimizer.tar'))
    assert st['t'] == 1 and st['dim'] == workload[0].D


def test_schedule_curriculum():
    cfg = C.Config(noise_stdev=0.1, batch_size=8, schedule_start=2, schedule_limit=3, stdev_divisor=2,
                   bs_multiplier=2)
    s = M.Schedule(cfg, 4)
    hits = []
    for _ in range(8):
        s.incr_iteration()
        hits.append(s.schedule_reached)
    # iteration.py:184-187: reached at it >= start and (it - start) % limit == 0 -> it = 2, 5, 8
    assert hits == [False, True, False, False, True, False, False, True]
    assert s.noise_stdev == 0.1 / 8 and s.batch_size == 64 and s.nb_samples_used == 8 + 8 + 16 * 3 + 32 * 3


class _Loader:
    """get_batch(split, batch_size) over a pool of images (the data.CocoFcDataLoader surface)."""

    def __init__(self, fc, gts):
        self.fc, self.gts, self.pos, self.sizes = fc, gts, 0, []

    def get_batch(self, split, batch_size=None):
        self.sizes.append(batch_size)
        ix = [(self.pos + k) % len(self.gts) for k in range(batch_size)]
        self.pos += batch_size
        return {'fc_feats': np.repeat(self.fc[ix], 5, axis=0), 'gts': [self.gts[i] for i in ix]}


def _sched_spec(P, bs, **cfg):
    base = {'noise_stdev': 0.05, 'batch_size': bs, 'l2coeff': 1e-3, 'snapshot_freq': 0}
    base.update(cfg)
    return C.ExperimentSpec(_exp(nb_offspring=P, config=base, policy_options={'net': 'fc_caption', 'fitness': 'greedy'},
                                 optimizer_options={'type': 'adam', 'args': {'stepsize': 0.01}}), vocab_size=63)


def test_curriculum_draws_batches_at_the_scheduled_size():
    """bs_multiplier (tools/iteration.py:149-153): with a loader the master asks for batches of the
    scheduled size, so a batch-size curriculum changes what is evaluated; stepsize_divisor applies."""
    dims, theta, fc, gts, df, n, table = tiny_workload(B=8)
    spec = _sched_spec(2, 2, schedule_start=1, schedule_limit=2, bs_multiplier=2, stepsize_divisor=4, single_batch=True)
    eng = OracleEngine(dims, theta, fc, gts, df, n, table)
    seen = []
    orig = eng.set_batch
    eng.set_batch = lambda f, g: (seen.append(len(g)), orig(f, g))
    loader = _Loader(fc, gts)
    m = M.EngineMaster(spec, eng)
    m.run(loader, max_iterations=4)
    # schedule reached at it = 1 and 3: the batch doubles after each
    assert loader.sizes == [2, 4, 4, 8] and seen == [2, 4, 4, 8]
    assert [r['batch_size'] for r in m.stats] == [4, 4, 8, 8]
    assert m.opt.stepsize == 0.01 / 16


def test_dispatched_loop_applies_the_schedule(workload, tmp_path):
    """run_dispatched divides the step size when the schedule is reached, as run() and
    the reference master (nic_nes_master.py:139-141) do; both loops end on the same theta."""
    dims, theta, fc, gts, df, n, table = workload
    P, iters = 4, 3
    batch = {'fc_feats': fc, 'gts': gts}
    cfg = dict(schedule_start=1, schedule_limit=2, stepsize_divisor=2)
    local = M.EngineMaster(_sched_spec(P, 4, **cfg), _engine(workload), log_dir=str(tmp_path / 'a'))
    local.run([batch] * iters, max_iterations=iters)
    master = M.EngineMaster(_sched_spec(P, 4, **cfg), _engine(workload), log_dir=str(tmp_path / 'b'))
    store = T.LocalStore()
    worker = N.EngineWorker(_engine(workload), _sched_spec(P, 4, **cfg), worker_id=1)
    th = threading.Thread(target=M.run_worker, args=(T.WorkerClient(store), worker),
                          kwargs=dict(chunk=4, max_tasks=iters), daemon=True)
    th.start()
    master.run_dispatched(T.MasterClient(store), [batch] * iters, max_iterations=iters, result_timeout=120)
    th.join(timeout=120)
    assert local.opt.stepsize == master.opt.stepsize == 0.01 / 4
    assert np.array_equal(local.e.theta()[0].numpy(), master.e.theta()[0].numpy())


def test_run_ends_on_an_exhausted_iterator(workload):
    """a one-shot iterator shorter than max_iterations ends the run instead of spinning."""
    import itertools
    dims, theta, fc, gts, df, n, table = workload
    m = M.EngineMaster(_spec(2), _engine(workload))
    stats = m.run(itertools.islice(iter([{'fc_feats': fc, 'gts': gts}] * 5), 2), max_iterations=5)
    assert len(stats) == 2 and m.sched.iteration == 2


def test_optimizer_file_is_reference_typed(workload, tmp_path):
    """optimizer.tar stores m, v as fp64 numpy arrays, the reference's types
    (optimizers.py:85-95)."""
    import pickle
    m = M.EngineMaster(_spec(2), _engine(workload), log_dir=str(tmp_path))
    m.run([{'fc_feats': workload[2], 'gts': workload[3]}], max_iterations=1)
    m.save_snapshot()
    # weights_only load with the numpy allowlist (what _load_state does): arrays come back as ndarrays
    import numpy.core.multiarray as ma
    with torch.serialization.safe_globals([ma._reconstruct, np.ndarray, np.dtype, type(np.dtype(np.float64))]):
        st = torch.load(str(tmp_path / 'snapshot' / 'optimizer.tar'), weights_only=True)
    assert isinstance(st['m'], np.ndarray) and st['m'].dtype == np.float64 and isinstance(st['v'], np.ndarray)
    assert pickle is not None


def test_set_batch_not_skipped_when_an_id_is_reused(workload):
    """A new batch whose dict reuses the id() of the freed previous one must still be loaded."""
    dims, theta, fc, gts, df, n, table = workload
    e = _engine(workload)
    loads = []
    orig = e.set_batch
    e.set_batch = lambda f, g: (loads.append(f.shape[0]), orig(f, g))
    m = M.EngineMaster(_spec(2), e)
    for k in range(3):
        m._set_batch({'fc_feats': fc[:k + 1], 'gts': gts[:k + 1]})       # each dict freed right after
    assert loads == [1, 2, 3]


def test_per_member_batches_single_batch_false():
    """single_batch false (mscoco_nes.json; nic_nes_worker.py:121-128 draws a batch per member): the
    master asks the loader for one batch per member (capped by batches_per_iteration) and member i
    is scored on batch i mod G, locally and through a dispatched worker alike."""
    dims, theta, fc, gts, df, n, table = tiny_workload(B=12)
    P = 4
    exp = _sched_spec(P, 3).exp
    exp['config']['single_batch'] = False
    exp['batches_per_iteration'] = 3
    spec = C.ExperimentSpec(exp, vocab_size=63)
    assert not spec.single_batch and spec.batches_per_iteration == 3
    eng = OracleEngine(dims, theta, fc, gts, df, n, table)
    loader = _Loader(fc, gts)
    m = M.EngineMaster(spec, eng)
    m.run(loader, max_iterations=1)
    assert loader.sizes == [3, 3, 3]
    # the fitness of member i is the one of batch i mod 3
    ref = OracleEngine(dims, theta, fc, gts, df, n, table)
    batches = [(fc[3 * g: 3 * g + 3], gts[3 * g: 3 * g + 3]) for g in range(3)]
    fit = np.zeros((P, 2))
    for i in range(P):
        ref.set_batch(*batches[i % 3])
        fit[i] = ref.evaluate(1, i, 1, 0.05).numpy()[0]
    rec = m.stats[0]
    assert rec['score_mean'] == float(fit.mean()) and rec['score_max'] == float(fit.max())
    # a worker handed the list of batches scores the same
    task = N.NESTask(batch_data=[{'fc_feats': b[0], 'gts': b[1]} for b in batches], noise_stdev=0.05, iteration=1)
    res = N.EngineWorker(OracleEngine(dims, theta, fc, gts, df, n, table), spec, worker_id=1).fitness_batch(1, task, 0, P)
    assert np.array_equal(np.stack([r.fitness for r in res]), fit)


# ------------------------------------------------------------------ safe / proportional mutations ----
def _mut_spec(P, mode, **mo):
    return C.ExperimentSpec(_exp(nb_offspring=P, config={'noise_stdev': 0.05, 'batch_size': 4, 'l2coeff': 1e-3,
                                                         'snapshot_freq': 0},
                                 policy_options={'net': 'fc_caption', 'fitness': 'greedy',
                                                 'model_options': dict(safe_mutations=mode, **mo)},
                                 optimizer_options={'type': 'adam', 'args': {'stepsize': 0.01}}), vocab_size=63)


def test_mutation_goldens_from_the_reference():
    """tests/golden/mutations.npz (scripts/make_golden.py, the reference's FCModel): the oracle's SM-G-SUM
    sensitivity (oracle/sensitivity_ref.py) equals Sensitivity.calc_sensitivity bit for bit; the oracle's transform of a noise draw
    equals PolicyNet.evolve's returned noise for SM-G-SUM and SM-PROPORTIONAL."""
    from nicnes import mutations as MU
    from oracle import sensitivity_ref as SR
    g = np.load('tests/golden/mutations.npz')
    V, E, R, F_ = [int(x) for x in g['dims']]
    s = MU.clamp_calc(SR.sum_sensitivity((V + 1, E, R, F_), g['theta'], g['fc'], 4), float(g['underflow']))
    assert np.array_equal(s.numpy(), g['sensitivity'])
    raw = g['raw']
    D = raw.size
    assert np.array_equal(O.member_delta(raw, 0, 1.0, D, ('divide', g['sensitivity'])), g['delta_safe'])
    prop = MU.proportional_vector(g['theta']).numpy()
    assert (g['theta'] == 0).sum() > 0 and np.array_equal(O.member_delta(raw, 0, 1.0, D, ('scale', prop)),
                                                          g['delta_prop'])


def test_mutation_vector_file(tmp_path):
    """Sensitivity.set_sensitivity (safe_mutations.py:27-31): clamp at the underflow, divide by the min."""
    from nicnes import mutations as MU
    v = torch.tensor([0.01, 0.5, 2.0, 0.05, 1.0])
    torch.save(v, str(tmp_path / 'sens.pt'))
    got = MU.load_vector_file(str(tmp_path / 'sens.pt'), 0.1)
    want = torch.tensor([0.1, 0.5, 2.0, 0.1, 1.0]) / 0.1
    assert torch.equal(got, want)


@pytest.mark.parametrize('mode', ['SM-G-SUM', 'SM-PROPORTIONAL'])
def test_mutation_dispatched_loop_matches_local_loop(workload, tmp_path, mode):
    """Workers (EngineWorker._prepare) and the master (_prepare_mutation) compute the same vector, so the
    dispatched loop's update equals the local loop's; and the mutation changes the trajectory."""
    dims, theta, fc, gts, df, n, table = workload
    P, iters = 4, 2
    batch = {'fc_feats': np.repeat(fc, 5, axis=0), 'gts': gts}
    spec = _mut_spec(P, mode, safe_mutation_underflow=0.1)
    local = M.EngineMaster(spec, _engine(workload), log_dir=str(tmp_path / 'a'))
    local.run([batch], max_iterations=iters)
    assert local.e.mutation is not None and local.e.mutation[0] == ('divide' if mode == 'SM-G-SUM' else 'scale')
    plain = M.EngineMaster(_spec(P), _engine(workload), log_dir=str(tmp_path / 'c'))
    plain.run([batch], max_iterations=iters)
    assert not np.array_equal(plain.e.theta()[0].numpy(), local.e.theta()[0].numpy())

    e_master, e_worker = _engine(workload), _engine(workload)
    master = M.EngineMaster(spec, e_master, log_dir=str(tmp_path / 'b'))
    store = T.LocalStore()
    worker = N.EngineWorker(e_worker, spec, worker_id=1)
    th = threading.Thread(target=M.run_worker, args=(T.WorkerClient(store), worker),
                          kwargs=dict(chunk=4, max_tasks=iters), daemon=True)
    th.start()
    master.run_dispatched(T.MasterClient(store), [batch] * iters, max_iterations=iters, result_timeout=120)
    th.join(timeout=120)
    assert not th.is_alive()
    assert np.array_equal(local.e.theta()[0].numpy(), master.e.theta()[0].numpy())
    assert np.array_equal(e_worker.mutation[1], e_master.mutation[1])


def test_epoch_counts_loader_wraps(workload):
    """A loader batch with bounds['wrapped'] ends an epoch (the reference re-enters its train loader,
    nic_nes_master.py:69-72); run_dispatched counts its own pass as one epoch."""
    dims, theta, fc, gts, df, n, table = workload

    class Wrapping:
        def __init__(self):
            self.k = 0

        def get_batch(self, split, batch_size=None):
            self.k += 1
            return {'fc_feats': np.repeat(fc, 5, axis=0), 'gts': gts, 'bounds': {'wrapped': self.k % 2 == 0}}
    spec = C.ExperimentSpec(_exp(nb_offspring=4, config={'noise_stdev': 0.05, 'batch_size': 4, 'l2coeff': 1e-3,
                                                         'snapshot_freq': 0, 'single_batch': True},
                                 policy_options={'net': 'fc_caption', 'fitness': 'greedy'},
                                 optimizer_options={'type': 'adam', 'args': {'stepsize': 0.01}}), vocab_size=63)
    m = M.EngineMaster(spec, _engine(workload))
    m.run(Wrapping(), max_iterations=4)
    assert m.sched.epoch == 1 + 2            # the run's own pass + wraps after batches 2 and 4


def test_mutation_worker_with_state_dict_models(workload):
    """EngineWorker with a mutation and tasks whose `current` is a state_dict (not a path): the per-task
    cache key must not compare tensors."""
    from nicnes import nes as NN
    dims, theta, fc, gts, df, n, table = workload
    e = _engine(workload)
    spec = _mut_spec(2, 'SM-PROPORTIONAL')
    w = N.EngineWorker(e, spec, worker_id=1)
    sd = NN.state_dict_from_vector(torch.from_numpy(theta), NN.param_shapes(e))
    batch = {'fc_feats': np.repeat(fc, 5, axis=0), 'gts': gts}
    for tid in (1, 2):
        res = w.fitness_batch(tid, N.NESTask(current=sd, batch_data=batch, noise_stdev=0.05, iteration=tid), 0, 2)
        assert len(res) == 2 and e.mutation[0] == 'scale'


def test_eval_rollouts_draw_a_fresh_stream_each(workload):
    """EnginePolicy.rollout (the eval result, CaptPolicy.rollout) hands nicnes_evaluate_theta a new draw iteration
    per call, as the reference worker's RNG draws afresh per eval (not iteration 0 every time)."""
    e = _engine(workload)
    seen = []
    orig = e.evaluate_theta

    def spy(batch=0, iteration=0, **kw):
        seen.append(iteration)
        return orig(batch, iteration=iteration)
    e.evaluate_theta = spy
    pol = N.EnginePolicy(e)
    data = {'fc_feats': np.repeat(workload[2], 5, axis=0), 'gts': workload[3]}
    pol.rollout(None, data, None)
    pol.rollout(None, data, None)
    s0 = pol._eval_salt
    assert seen == [(s0 + 1) & 0xffffffff, (s0 + 2) & 0xffffffff]     # this process's salt + the call count


class _FaultingEngine(OracleEngine):
    """The oracle engine with the HIP engine's contained-fault contract: the first `faults` optimizer steps
    raise DecodeFault and change nothing (the device skips them); clear_faults reports and clears."""

    def __init__(self, *a, faults=1, **k):
        super().__init__(*a, **k)
        self.faults_left, self.cleared = faults, 0

    def adam_step(self, *a, **k):
        if self.faults_left > 0:
            self.faults_left -= 1
            from nicnes import DecodeFault
            raise DecodeFault('adam_step failed: contained decode fault: coop decode: hand-off timeout')
        return super().adam_step(*a, **k)

    def clear_faults(self):
        self.cleared += 1
        return {'coop_timeouts': 1, 'sample_slot_timeouts': 0}


def test_master_reruns_a_contained_fault(workload, tmp_path):
    """EngineMaster.run: a faulted iteration is recorded, the handle cleared and the same
    iteration re-run, ending as the unfaulted run; past fault_retries a snapshot is written and the fault raised."""
    import nicnes
    dims, theta, fc, gts, df, n, table = workload
    P = 4
    ref_e = OracleEngine(dims, theta, fc, gts, df, n, table)
    ref = M.EngineMaster(_spec(P), ref_e, log_dir=str(tmp_path / 'ref'))
    ref.run([(fc, gts)] * 3, max_iterations=3)
    e = _FaultingEngine(dims, theta, fc, gts, df, n, table, faults=1)
    m = M.EngineMaster(_spec(P), e, log_dir=str(tmp_path / 'f1'))
    m.run([(fc, gts)] * 3, max_iterations=3, fault_retries=1)
    assert e.cleared == 1 and [(f['iter'], f['attempt']) for f in m.faults] == [(1, 0)]
    assert (tmp_path / 'f1' / 'faults' / 'fault_i1_a0.json').exists()
    assert [s['score_mean'] for s in m.stats] == [s['score_mean'] for s in ref.stats]
    assert np.array_equal(e.adam.theta, ref_e.adam.theta)
    e2 = _FaultingEngine(dims, theta, fc, gts, df, n, table, faults=2)
    m2 = M.EngineMaster(_spec(P), e2, log_dir=str(tmp_path / 'f2'))
    with pytest.raises(nicnes.DecodeFault):
        m2.run([(fc, gts)] * 3, max_iterations=3, fault_retries=1)
    assert [(f['iter'], f['attempt']) for f in m2.faults] == [(1, 0), (1, 1)] and m2.stats == []
    # the snapshot records the state before the faulted iteration 1 (iteration 0), theta / m / v included
    assert list((tmp_path / 'f2' / 'snapshot').glob('z_info_e1_i0-0.json'))


def test_fault_snapshot_at_a_schedule_boundary_records_the_pre_fault_schedule(workload, tmp_path):
    """when the faulted iteration is a curriculum boundary, incr_iteration has already divided sigma and
    grown the batch; the fault snapshot must hold the schedule as it was before (matching theta, m, v), i.e. equal
    the snapshot an unfaulted run writes after the previous iteration, so resuming does not step the curriculum
    twice."""
    import json as _json
    import nicnes
    dims, theta, fc, gts, df, n, table = workload
    P = 4
    cfg = dict(schedule_start=1, schedule_limit=2, stdev_divisor=2, bs_multiplier=2)   # boundaries at it = 1, 3
    ref = M.EngineMaster(_sched_spec(P, 4, **cfg), OracleEngine(dims, theta, fc, gts, df, n, table),
                         log_dir=str(tmp_path / 'ref'))
    ref.run([(fc, gts)] * 2, max_iterations=2)
    want = _json.loads(open(ref.save_snapshot()).read())
    e = _FaultingEngine(dims, theta, fc, gts, df, n, table, faults=0)
    m = M.EngineMaster(_sched_spec(P, 4, **cfg), e, log_dir=str(tmp_path / 'f'))
    m.run([(fc, gts)] * 2, max_iterations=2)
    e.faults_left = 2                                   # iteration 3 (a boundary) faults on both tries
    with pytest.raises(nicnes.DecodeFault):
        m.run([(fc, gts)] * 2, max_iterations=3, fault_retries=1)
    [snap] = list((tmp_path / 'f' / 'snapshot').glob('z_info_*.json'))
    got = _json.loads(snap.read_text())
    for k in ('iter', 'noise_stdev', 'batch_size', 'times_orig_bs', 'nb_samples_used', 'bad_generations'):
        assert got[k] == want[k], k
    assert got['noise_stdev'] == 0.05 / 2 and got['iter'] == 2
    # resuming replays the schedule exactly as the unfaulted run's snapshot would
    r = M.Schedule(_sched_spec(P, 4, **cfg).config, P)
    r.init_from_infos(got)
    r.incr_iteration()
    ref.sched.init_from_infos(want)
    ref.sched.incr_iteration()
    a, b = r.to_dict(), ref.sched.to_dict()
    a.pop('epoch'), b.pop('epoch')                       # the faulted master ran two passes (two run() calls)
    assert a == b


def test_eval_rollout_draw_streams_differ_between_processes(workload):
    """two workers sharing --noise_seed (or a restarted worker) must not replay each other's eval
    draws. Each EnginePolicy starts its eval stream at a random 32-bit salt (the engine hashes the low 32 bits
    of the iteration), then steps by one per rollout."""
    dims, theta, fc, gts, df, n, table = workload
    seen = []

    class _Rec(OracleEngine):
        def evaluate_theta(self, batch=0, iteration=0):
            seen.append(iteration)
            return super().evaluate_theta(batch, iteration)

    pa = N.EnginePolicy(_Rec(dims, theta, fc, gts, df, n, table))
    pb = N.EnginePolicy(_Rec(dims, theta, fc, gts, df, n, table))
    batch = {'fc_feats': np.repeat(fc, 5, axis=0), 'gts': gts}
    for p in (pa, pb, pa):
        p.rollout(None, batch, None)
    assert seen[0] != seen[1]                               # two processes' first eval draws
    assert seen[2] == (seen[0] + 1) & 0xffffffff            # the next rollout of the same process
    assert all(0 <= s < 2 ** 32 for s in seen)
