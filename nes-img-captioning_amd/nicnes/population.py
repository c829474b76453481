"""One NIC-NES iteration over a population, sharded over the ranks of a torch.distributed group.

Replaces the master/worker split of the reference for the hot path:
  workers: NESWorker.fitness per member            (/root/reference/src/algorithm/nic_nes/nic_nes_worker.py:115-161)
  master : gradient_estimate + optimizer.update     (/root/reference/src/algorithm/nic_nes/nic_nes_master.py:123-137)
with members [r*P/N, (r+1)*P/N) evaluated on rank r. The exchange is one all-gather of the (P, 2)
fitness (every rank then ranks the whole population identically) and one all-reduce (sum) of the
D-float weighted noise sum; Adam then runs replicated, so theta needs no broadcast.
Two bindings of the exchange: torch.distributed (comm=None; on ROCm the 'nccl' backend is RCCL over
xGMI, 'gloo' on CPU), or the engine's own C-ABI RCCL communicator (comm='engine':
nicnes_allgather_fitness / nicnes_allreduce_grad after Engine.comm_init), for callers that do not
run torch.distributed.
"""
import torch
import torch.distributed as dist


class PopulationRunner:
    """Per iteration both bindings issue the same two collectives: one all-gather of the fitness and ONE
    all-reduce of the noise sum (north_star's single all-reduce).
    overlap_chunks > 1 (opt-in, torch.distributed exchange, world > 1; unmeasured on hardware): the noise
    sum is computed in that many parameter ranges, each range's all-reduce running on the collective stream
    while the next range is summed -- that many all-reduces per iteration instead of one."""

    def __init__(self, engine, population, sigma, l2coeff=0.0, stepsize=1e-3, beta1=0.9, beta2=0.999,
                 epsilon=1e-08, rank=0, world_size=1, group=None, comm=None, overlap_chunks=1):
        assert population % world_size == 0, 'population must split evenly over ranks'
        self.e = engine
        self.P = population
        self.sigma = float(sigma)
        self.l2coeff, self.stepsize, self.beta1, self.beta2, self.epsilon = l2coeff, stepsize, beta1, beta2, epsilon
        self.rank, self.world = rank, world_size
        self.group = group
        if comm not in (None, 'engine'):
            raise ValueError("comm: None (torch.distributed) or 'engine' (the engine's RCCL communicator)")
        self.comm = comm
        self.local = population // world_size
        self.m0 = rank * self.local
        dev = engine.device
        self.fit_local = torch.empty((self.local, 2), dtype=torch.float64, device=dev)
        self.fit_all = torch.empty((self.P, 2), dtype=torch.float64, device=dev) if world_size > 1 else self.fit_local
        self.gsum = torch.empty(engine.D, dtype=torch.float32, device=dev)
        D = engine.D
        n = max(1, int(overlap_chunks)) if (world_size > 1 and comm is None and
                                             hasattr(engine, 'grad_partial_range')) else 1
        cuts = [0] + [min(D, (D * k // n + 63) // 64 * 64) for k in range(1, n)] + [D]
        self.ranges = [(a, b) for a, b in zip(cuts[:-1], cuts[1:]) if b > a]

    def evaluate(self, iteration, n_batches=1):
        """this rank's members -> fitness [local, 2] (f+, f-). With n_batches > 1 (the engine holds
        that many batches, single_batch: false) member i is scored on batch i mod n_batches."""
        mb = None if n_batches <= 1 else [(self.m0 + k) % n_batches for k in range(self.local)]
        if mb is None:
            self.e.evaluate(iteration, self.m0, self.local, self.sigma, fitness_out=self.fit_local)
        else:
            self.e.evaluate(iteration, self.m0, self.local, self.sigma, fitness_out=self.fit_local, member_batch=mb)
        return self.fit_local

    def exchange_fitness(self):
        if self.world > 1:
            if self.comm == 'engine':
                self.e.allgather_fitness(self.fit_local, self.fit_all)
            else:
                dist.all_gather_into_tensor(self.fit_all, self.fit_local, group=self.group)
        return self.fit_all

    def reduce_noise_sum(self):
        if self.world > 1:
            if self.comm == 'engine':
                self.e.allreduce_grad(self.gsum)
            else:
                dist.all_reduce(self.gsum, op=dist.ReduceOp.SUM, group=self.group)
        return self.gsum

    def update(self, iteration, sync=True):
        """ranks -> weighted noise sum (local members) -> all-reduce -> Adam. Returns the update ratio
        (sync=False: nothing waits for the GPU and None is returned; engine.last_ratio() reads it)."""
        _, w = self.e.rank_weights(self.fit_all)
        w_local = w[self.m0:self.m0 + self.local]
        if len(self.ranges) > 1:
            # range k's all-reduce (collective stream) overlaps the sum of range k + 1 (compute stream)
            works = []
            for j0, j1 in self.ranges:
                self.e.grad_partial_range(iteration, self.m0, self.local, w_local, self.sigma, j0, j1, self.gsum)
                works.append(dist.all_reduce(self.gsum[j0:j1], op=dist.ReduceOp.SUM, group=self.group,
                                             async_op=True))
            for wk in works:
                wk.wait()
        else:
            self.e.grad_partial(iteration, self.m0, self.local, w_local, self.sigma, out=self.gsum)
            self.reduce_noise_sum()
        return self.e.adam_step(self.gsum, self.P, self.l2coeff, self.stepsize, self.beta1, self.beta2,
                                self.epsilon, sync=sync)

    def step(self, iteration, sync=True, n_batches=1):
        """One full NES iteration. Returns (fitness [P, 2] on device, update ratio). With sync=False the
        iteration is only enqueued (ratio None): back-to-back iterations then keep the GPU busy, so
        its clock does not drop between them. n_batches > 1: per-member batches (evaluate)."""
        self.evaluate(iteration, n_batches)
        self.exchange_fitness()
        ratio = self.update(iteration, sync=sync)
        return self.fit_all, ratio
