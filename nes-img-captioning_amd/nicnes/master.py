"""The NIC-NES master loop and the engine worker loop.

  Schedule             Iteration's noise/batch curriculum (/root/reference/src/algorithm/tools/iteration.py:16-192)
  EngineMaster.run     NESMaster.run_master, single node, sharded over torch.distributed ranks
                       (/root/reference/src/algorithm/nic_nes/nic_nes_master.py:56-168)
  EngineMaster.run_dispatched
                       the same loop over the redis-style transport: declare NESTask, pop NESResults
                       of the current task, gradient_estimate + optimizer.update (nic_nes_master.py:80-137)
  run_worker           NESWorker.run_worker for the engine (nic_nes_worker.py:40-97): claims member
                       chunks of the current task and pushes one NESResult per member
  save_snapshot        theta .pth + optimizer.tar + z_info json (/root/reference/src/algorithm/tools/snapshot.py:14-38,
                       optimizers.py:85-107)
Validation-set evaluation, elites/podium and plotting are outside the engine's scope.
"""
import json
import os
import re
import time

import numpy as np
import torch

from .nes import NESTask, make_optimizer, state_dict_from_vector, param_shapes, EnginePolicy, engine_batch
from .population import PopulationRunner


class Schedule:
    """Noise-stdev / batch-size curriculum with the reference's counters and to_dict keys."""

    def __init__(self, config, nb_offspring):
        self.noise_stdev = float(config.noise_stdev)
        self.batch_size = int(config.batch_size)
        self.times_orig_bs = 1
        self.nb_samples_used = 0
        self.bad_generations = 0
        self.epoch = 0
        self.iteration = 0
        self.schedule_limit = config.schedule_limit
        self.schedule_start = config.schedule_start or 0
        self.stdev_divisor = config.stdev_divisor or 1.0
        self.bs_multiplier = config.bs_multiplier or 1.0
        self.patience = config.patience
        self.nb_offspring = int(nb_offspring)
        self.schedule_reached = False

    def incr_iteration(self):
        """iteration.py:165-182"""
        self.schedule_reached = False
        self.iteration += 1
        self.nb_samples_used += self.batch_size
        if self.check_schedule_limit():
            self.schedule_reached = True
            self.next_curriculum_step()

    def check_schedule_limit(self):
        return bool(self.schedule_limit) and self.iteration >= self.schedule_start and \
            (self.iteration - self.schedule_start) % self.schedule_limit == 0

    def next_curriculum_step(self):
        """iteration.py:149-153"""
        self.noise_stdev /= self.stdev_divisor
        self.batch_size = int(self.batch_size * self.bs_multiplier)
        self.times_orig_bs *= self.bs_multiplier

    def to_dict(self):
        return {'iter': self.iteration, 'epoch': self.epoch, 'noise_stdev': self.noise_stdev,
                'batch_size': self.batch_size, 'bad_generations': self.bad_generations,
                'times_orig_bs': self.times_orig_bs, 'nb_samples_used': self.nb_samples_used}

    def init_from_infos(self, infos):
        """iteration.py:60-75 (iter/epoch are stored post-increment)."""
        self.epoch = infos.get('epoch', self.epoch + 1) - 1
        self.iteration = infos.get('iter', self.iteration + 1) - 1
        for k in ('bad_generations', 'noise_stdev', 'batch_size', 'times_orig_bs', 'nb_samples_used'):
            if k in infos:
                setattr(self, k, infos[k])


class EngineMaster:
    def __init__(self, spec, engine, log_dir=None, rank=0, world_size=1, group=None, theta=None, comm=None):
        self.spec, self.e = spec, engine
        self.log_dir = log_dir or spec.config.log_dir or 'logs/nicnes'
        self.rank, self.world, self.group, self.comm = rank, world_size, group, comm
        self.sched = Schedule(spec.config, spec.nb_offspring)
        self.policy = EnginePolicy(engine, spec)
        if theta is not None:
            engine.set_theta(theta)
        self.opt = make_optimizer(engine, spec)
        self.stats = []
        self.faults = []
        self._batch_key = None
        self._n_batches = 1
        self.mutator = None
        if spec.mutation:
            from .mutations import Mutator
            self.mutator = Mutator(spec, engine)

    def _prepare_mutation(self, batch):
        """Safe / proportional mutations: the iteration's noise transform, computed from the fp32 theta
        the members evaluate and the iteration's (first) batch, the vector the workers compute
        (nicnes.mutations)."""
        if self.mutator is not None and self.mutator.active:
            from .mutations import batch_fc
            self.mutator.prepare(self.sched.iteration, lambda: self.e.theta()[1], batch_fc(batch))

    # ------------------------------------------------------------------------ helpers ----------
    def _set_batch(self, batch):
        """One batch (dict, or (fc, gts)) shared by every member, or a list of G batches (single_batch:
        false: member i uses batch i mod G). The batch object itself is kept: an id() of a freed batch
        can be reused by the next one."""
        if batch is not self._batch_key:
            if isinstance(batch, list):
                ub = [engine_batch(b, self.e) if isinstance(b, dict) else b for b in batch]
                if len(ub) == 1:
                    self.e.set_batch(*ub[0])
                else:
                    self.e.set_batches(ub)
                self._n_batches = len(ub)
            else:
                fc, gts = engine_batch(batch, self.e) if isinstance(batch, dict) else batch
                self.e.set_batch(fc, gts)
                self._n_batches = 1
            self._batch_key = batch

    def _update(self, gsum, P):
        return self.opt.update_from_noise_sum(gsum, P, self.spec.l2coeff)

    def _record(self, fit, ratio, t0):
        f = fit.detach().cpu().numpy() if isinstance(fit, torch.Tensor) else np.asarray(fit)
        rec = {'iter': self.sched.iteration, 'update_ratio': float(ratio), 'score_mean': float(f.mean()),
               'score_max': float(f.max()), 'score_min': float(f.min()), 'noise_stdev': self.sched.noise_stdev,
               'batch_size': self.sched.batch_size, 'step_time': time.time() - t0}
        self.stats.append(rec)
        return rec

    def _maybe_snapshot(self):
        freq = self.spec.config.snapshot_freq
        if self.rank == 0 and freq and self.sched.iteration % freq == 0:
            self.save_snapshot()

    def _after_update(self):
        """nic_nes_master.py:139-141,161-163: when the schedule is reached the Adam step size is
        divided by stepsize_divisor (the noise / batch curriculum already moved in incr_iteration)."""
        if self.sched.schedule_reached and self.spec.config.stepsize_divisor:
            self.opt.stepsize /= self.spec.config.stepsize_divisor

    def _batch_stream(self, batches):
        """Yield one batch per iteration. A loader (an object with get_batch, e.g. data.CocoFcDataLoader)
        is asked for batches of the CURRENT scheduled size, so a bs_multiplier curriculum changes what
        is evaluated (the reference restarts its loader with the new size, tools/iteration.py:150-154);
        any other iterable is consumed as given, one pass per epoch."""
        if hasattr(batches, 'get_batch'):
            G = self.spec.batches_per_iteration
            while True:
                if G == 1:
                    got = [batches.get_batch('train', batch_size=self.sched.batch_size)]
                else:          # single_batch: false -- one batch per member (nic_nes_worker.py:121-128)
                    got = [batches.get_batch('train', batch_size=self.sched.batch_size) for _ in range(G)]
                # a loader that wrapped around its split ends an epoch (the reference's outer loop,
                # nic_nes_master.py:69-72, re-enters its train loader then)
                if any(isinstance(b, dict) and b.get('bounds', {}).get('wrapped') for b in got):
                    self.sched.epoch += 1
                yield got[0] if G == 1 else got
        for b in batches:
            yield b

    # ------------------------------------------------------------------------ loops ------------
    def _iterate(self, runner, P):
        """One iteration on the current batch: evaluate this rank's shard, exchange, noise sum, update."""
        runner.evaluate(self.sched.iteration, n_batches=self._n_batches)
        fit = runner.exchange_fitness()
        _, w = self.e.rank_weights(fit)
        self.e.grad_partial(self.sched.iteration, runner.m0, runner.local,
                            w[runner.m0:runner.m0 + runner.local], self.sched.noise_stdev, out=runner.gsum)
        runner.reduce_noise_sum()
        return fit, self._update(runner.gsum, P)

    def _record_fault(self, err, attempt, counters):
        rec = {'iter': self.sched.iteration, 'attempt': attempt, 'error': str(err), **counters,
               'time': time.time()}
        self.faults.append(rec)
        if self.rank == 0:
            d = os.path.join(self.log_dir, 'faults')
            os.makedirs(d, exist_ok=True)
            with open(os.path.join(d, 'fault_i%d_a%d.json' % (self.sched.iteration, attempt)), 'w') as f:
                json.dump(rec, f)
        return rec

    def run(self, batches, max_iterations=None, fault_retries=1):
        """Single-node loop: every rank evaluates its shard of the population; one all-gather of the
        fitness and one all-reduce of the noise sum per iteration (population.py). `batches`: a loader
        (batches drawn at the scheduled batch size) or an iterable of batches, re-iterated per epoch;
        an iterable that yields nothing ends the run.

        Contained decode faults (nicnes.DecodeFault: a coop hand-off or logit-slot timeout) cost no state:
        the faulted iteration's fitness is NaN on every rank and its optimizer step is skipped everywhere,
        so theta / m / v / t are those before it. The iteration is recorded (self.faults, and
        <log_dir>/faults/ on rank 0), the handle's fault counters cleared, and the same iteration (same
        members, noise indices and batch) re-run, up to `fault_retries` times; after that a snapshot of
        the pre-fault state is written (rank 0) and the DecodeFault propagates, so the process exits
        non-zero with a resumable snapshot instead of a half-finished run. The reference has no such
        path: a dead worker process is restarted and the master waits (main.py:107-141)."""
        from ._lib import DecodeFault
        P = self.spec.nb_offspring
        max_it = max_iterations or self.spec.config.max_nb_iterations
        runner = None
        while not max_it or self.sched.iteration < max_it:
            self.sched.epoch += 1
            yielded = False
            for batch in self._batch_stream(batches):
                yielded = True
                t0 = time.time()
                before = dict(self.sched.__dict__)      # the schedule a fault snapshot must record
                self.sched.incr_iteration()
                self._set_batch(batch)
                self._prepare_mutation(batch)
                if runner is None or runner.sigma != self.sched.noise_stdev:
                    runner = PopulationRunner(self.e, P, self.sched.noise_stdev, rank=self.rank,
                                              world_size=self.world, group=self.group, comm=self.comm)
                for attempt in range(int(fault_retries) + 1):
                    try:
                        fit, ratio = self._iterate(runner, P)
                        break
                    except DecodeFault as err:
                        self._record_fault(err, attempt, self.e.clear_faults())
                        if attempt == int(fault_retries):
                            # theta / m / v are those before the faulted iteration, so the snapshot records the
                            # schedule as it was then too (a curriculum step taken by incr_iteration undone):
                            # resuming from it replays the faulted iteration exactly once
                            self.sched.__dict__.update(before)
                            if self.rank == 0:
                                self.save_snapshot()
                            raise
                self._record(fit, ratio, t0)
                self._after_update()
                self._maybe_snapshot()
                if max_it and self.sched.iteration >= max_it:
                    return self.stats
                if self.sched.schedule_reached and not hasattr(batches, 'get_batch'):
                    break          # batch size changed: the caller's iterable yields new batches
            if not yielded:
                return self.stats  # an exhausted one-shot iterator: nothing more to evaluate
        return self.stats

    def current_model_path(self):
        d = os.path.join(self.log_dir, 'models', 'current')
        os.makedirs(d, exist_ok=True)
        return os.path.join(d, '0_current_params.pth')

    def serialize_current(self):
        """theta as a state_dict .pth: fp32 before the first update, the fp64 master after (fact 8)."""
        t64, t32 = self.e.theta()
        vec = t32 if self.opt.t == 0 else t64
        path = self.current_model_path()
        torch.save(state_dict_from_vector(vec, param_shapes(self.e)), path)
        return path

    def run_dispatched(self, client, batches, max_iterations=1, result_timeout=600.0):
        """Master side over the transport (MasterClient). Members are ids [0, P) handed out by the
        per-task counter; results of stale tasks and surplus ids are dropped, as the reference drops
        results whose task_id is not current (nic_nes_master.py:108-116)."""
        P = self.spec.nb_offspring
        client.declare_experiment(self.spec.exp)
        self.sched.epoch += 1                   # it.incr_epoch() before the pass (nic_nes_master.py:70)
        done = 0
        for batch in self._batch_stream(batches):
            if done >= max_iterations:
                break
            t0 = time.time()
            self.sched.incr_iteration()
            self._set_batch(batch)
            self._prepare_mutation(batch)
            sigma = self.sched.noise_stdev
            task_id = client.declare_task(NESTask(current=self.serialize_current(), batch_data=batch,
                                                  noise_stdev=sigma, batch_size=self.sched.batch_size,
                                                  iteration=self.sched.iteration))
            fit = np.full((P, 2), np.nan)
            got = 0
            deadline = time.time() + result_timeout
            while got < P:
                tid, res = client.pop_result(timeout=max(deadline - time.time(), 0.001))
                if tid is None:
                    raise TimeoutError('%d of %d members arrived for task %d' % (got, P, task_id))
                if tid != task_id or res.fitness is None or res.member is None or res.member >= P:
                    continue
                if np.isnan(fit[res.member, 0]):
                    got += 1
                fit[res.member] = res.fitness
            fit_t = torch.from_numpy(fit).to(self.e.device)
            _, w = self.e.rank_weights(fit_t)
            gsum = self.e.grad_partial(self.sched.iteration, 0, P, w, sigma)
            ratio = self._update(gsum, P)
            self._record(fit, ratio, t0)
            self._after_update()
            self._maybe_snapshot()
            done += 1
        return self.stats

    # ------------------------------------------------------------------------ snapshots --------
    def save_snapshot(self):
        d = os.path.join(self.log_dir, 'snapshot')
        os.makedirs(d, exist_ok=True)
        theta_path = self.serialize_current()
        self.opt.save_to_file(os.path.join(d, 'optimizer.tar'))
        for f in os.listdir(d):
            if re.match(r'z_info_e[0-9]*?_i[0-9]*?-[0-9]*?.json', f):
                os.remove(os.path.join(d, f))
        infos = {**self.sched.to_dict(), 'current_model': theta_path,
                 'optimizer_state': os.path.join(d, 'optimizer.tar'), 'stats': self.stats[-1:] or []}
        name = 'z_info_e{e}_i{i}-{n}.json'.format(e=self.sched.epoch, i=self.sched.iteration, n=0)
        with open(os.path.join(d, name), 'w') as f:
            json.dump(infos, f)
        return os.path.join(d, name)

    def load_snapshot(self, info_path):
        with open(info_path) as f:
            infos = json.load(f)
        self.sched.init_from_infos(infos)
        self.policy.set_model(infos['current_model'])
        if os.path.exists(infos.get('optimizer_state', '')):
            self.opt.load_from_file(infos['optimizer_state'])
        return infos


def run_worker(client, worker, chunk=64, max_tasks=None, stop=None, idle_sleep=0.005):
    """Evaluate chunks of members of the current task until `max_tasks` tasks were seen or `stop`
    (a threading.Event) is set. Chunks beyond the population are still evaluated and dropped by the
    master, as surplus reference results are."""
    seen = set()
    while not (stop is not None and stop.is_set()):
        task_id, task = client.get_current_task()
        seen.add(task_id)
        begin = client.claim_members(task_id, chunk)
        P = getattr(worker.spec, 'nb_offspring', None) if worker.spec is not None else None
        count = chunk if P is None else max(min(chunk, P - begin), 0)
        if count == 0:
            if max_tasks is not None and len(seen) >= max_tasks:
                return len(seen)
            time.sleep(idle_sleep)
            continue
        client.push_results(task_id, worker.fitness_batch(task_id, task, begin, count))
    return len(seen)
