#!/usr/bin/env python3
"""Benchmark: NIC-NES population members evaluated per second (fc_caption), BASELINE.json's metric.

One step = one full NES iteration over the population on synthetic inputs resident in HBM:
perturb (in LDS) + greedy decode of both antithetic candidates of every member + CIDEr-D fitness,
fitness all-gather, centred ranks, weighted noise sum, gradient all-reduce, Adam.
Workload (BASELINE.json metric, 'fc_caption, pop=512 ... at 1/2/4/8 GPUs'; configs[2] at N = 1):
a population of 512 members, 128 unique images, sigma 0.01, l2coeff 1e-7, Adam 1e-3.
Multi-GPU is STRONG scaling by default, as the reference scales: more workers split a fixed
nb_offspring (main.py:105,144-153; tools/iteration.py:173; the master waits for nb_offspring results,
nic_nes_master.py:92-118), so rank r evaluates members [r P/N, (r+1) P/N) of the same P = 512.
--preset names the other BASELINE configs: configs1 (pop=64), configs3 (pop=2048; 256 per GPU on 8),
configs4 ('bu' features, pop=512; 64 per GPU on 8). --pop-per-gpu M is weak scaling (P = M N).

    python bench.py [--gpus N --steps K --warmup W] [--preset metric|configs1|configs2|configs3|configs4]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

--gpus N without a launcher (no WORLD_SIZE in the environment) starts N rank processes itself, before
anything touches the GPU, with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT set
as torch.distributed.run sets them, and exits with the first failing rank's status. Under a launcher
--gpus must equal WORLD_SIZE (exit 2 otherwise: a one-GPU number is never printed as an N-GPU one).
The line records what the collective saw (dist.get_world_size(); ncclCommCount with --comm engine) and
every rank's member range and decode / exchange / update times.
"""
import hashlib
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, 'nes-img-captioning_amd'))

METRIC = 'population-members evaluated/sec (fc_caption, pop=512) at 1/2/4/8 GPUs'
FP32_MFMA_PEAK_TFLOPS = 157.3       # MI355X dense fp32 MFMA (MI355X_MICROARCH.md, chip table)
HBM_PEAK_GBS = 8000.0


def decode_flops_per_member(B, V1=9488, E=128, R=128, F=2048):
    """Algorithmic FLOPs of one member (2 decodes of B unique rows): img_embed once, 17 cell
    steps, 16 logit steps per row."""
    per_row = 2 * (F * E + 17 * (2 * E * 5 * R) + 16 * (R * V1))
    return 2 * B * per_row


def step_noise_bytes_per_member(B, T=16, V1=9488, E=128, R=128):
    """Algorithmic HBM bytes of one member over the T + 2 step launches of a decode: the member's own
    noise rows, read once per use (they cannot stay on chip between steps): the logit matrix + bias
    at each of the T logit steps, the i2h/h2h matrices + biases at each of the T + 1 cells, and the
    2 x B embedding rows of each step's tokens (T - 1 token steps; the BOS step reads one row).
    Base theta is shared by every member (L2/MALL) and not counted."""
    logit = V1 * (R + 1) * 4
    cell = 2 * 5 * R * (E + 1) * 4
    emb = 2 * B * E * 4
    return T * logit + (T + 1) * cell + (T - 1) * emb + E * 4


def step_flops_per_member(B, V1=9488, E=128, R=128):
    """The part of decode_flops_per_member done by nicnes_decode_step_kernel: the 16 logit GEMMs and
    the 17 LSTM cells' gate sums, i2h and h2h halves (the img kernel does the image projection)."""
    per_row = 2 * (17 * (2 * E * 5 * R) + 16 * (R * V1))
    return 2 * B * per_row


def logit_flops_per_member(B, V1=9488, R=128, T=16):
    """The logit GEMMs of one member (2 decodes of B rows, T steps): the split path's logit kernel."""
    return 2 * B * T * 2 * R * V1


def logit_noise_bytes_per_member(V1=9488, R=128):
    """A member's logit-matrix + bias noise rows, read once per logit launch."""
    return V1 * (R + 1) * 4


def iteration_algorithmic_bytes(B, P, D=2865808):
    """HBM bytes one iteration must move per GPU: every member's noise rows at each
    decode step (step_noise_bytes_per_member), its noise slice once more for the weighted sum, the
    weighted sum written once, and Adam's fp64 theta / m / v read + written with g read and theta32
    written."""
    return P * (step_noise_bytes_per_member(B) + 4 * D) + 4 * D + (3 * 2 * 8 + 4 + 4) * D


# BASELINE.json configs by name: (population, batch, bu features, the config's text)
PRESETS = {
    'metric': (512, 128, False, 'the metric: fc_caption pop=512 at 1/2/4/8 GPUs (configs[2] at N = 1)'),
    'configs1': (64, 128, False, 'configs[1]: mscoco_nes.json fc_caption, synthetic 2048-d fc feats, pop=64'),
    'configs2': (512, 128, False, 'configs[2]: mscoco_nes.json fc_caption, pop=512 antithetic, batch_size=128'),
    'configs3': (2048, 128, False, 'configs[3]: mscoco_nes.json fc_caption, pop=2048 sharded (256 per GPU on 8)'),
    'configs4': (512, 128, True, "configs[4]: mscoco_nes.json with 'bu' features, pop=512 (64 per GPU on 8)"),
}

# committed PMC profiles: profiles/<round>_pmc_<key>_p<members per GPU>_b<B>.json
PMC_KEYS = {'nicnes_decode_steps_kernel': 'steps', 'nicnes_decode_step_kernel': 'step',
            'nicnes_decode_logit_kernel<4>': 'logit', 'nicnes_decode_coop_kernel<4>': 'coop4',
            'nicnes_decode_coop_kernel<2>': 'coop2', 'nicnes_decode_steps2_kernel': 'steps2',
            'nicnes_decode_steps_kernel<sample>': 'sampled'}
KERNEL_SOURCES = ('nes-img-captioning_amd/csrc/decode_kernel.hip', 'nes-img-captioning_amd/csrc/decode_kernel.h',
                  'include/nicnes_math.h')


def kernel_source_sha256():
    """Hash of the decode kernel's sources: a PMC profile records it, and bench.py uses the profile's
    counter figures only while the sources still hash the same."""
    h = hashlib.sha256()
    for f in KERNEL_SOURCES:
        with open(os.path.join(REPO, f), 'rb') as fh:
            h.update(fh.read())
    return h.hexdigest()


# the instantiation a PMC key names: (key, PAIRS) -> mangled symbol (PAIRS: the greedy-only bounded-lse variant)
PMC_SYMBOLS = {
    ('steps', True): '_Z26nicnes_decode_steps_kernelILb1ELb0EEv12DecodeParams',
    ('steps', False): '_Z26nicnes_decode_steps_kernelILb0ELb0EEv12DecodeParams',
    ('sampled', False): '_Z26nicnes_decode_steps_kernelILb0ELb1EEv12DecodeParams',
    ('coop4', True): '_Z25nicnes_decode_coop_kernelILb1ELi4EEv12DecodeParamsi',
    ('coop4', False): '_Z25nicnes_decode_coop_kernelILb0ELi4EEv12DecodeParamsi',
    ('coop2', True): '_Z25nicnes_decode_coop_kernelILb1ELi2EEv12DecodeParamsi',
    ('coop2', False): '_Z25nicnes_decode_coop_kernelILb0ELi2EEv12DecodeParamsi',
    ('steps2', True): '_Z27nicnes_decode_steps2_kernelILb1EEv12DecodeParams',
    ('steps2', False): '_Z27nicnes_decode_steps2_kernelILb0EEv12DecodeParams',
    ('logit', True): '_Z26nicnes_decode_logit_kernelILi4ELb1EEv12DecodeParamsi',
    ('logit', False): '_Z26nicnes_decode_logit_kernelILi4ELb0EEv12DecodeParamsi',
}
LIBRARY = os.path.join(REPO, 'nes-img-captioning_amd', 'nicnes', 'libnicnes.so')
_listings = {}


def library_kernel_sha(symbol, library=LIBRARY):
    """SHA-256 of the symbol's machine code in the library this run loads (nicnes.codeobj)."""
    from nicnes import codeobj
    if library not in _listings:
        _listings[library] = codeobj.kernel_listings(library)
    return codeobj.kernel_isa_sha256(library, symbol, _listings[library])


def load_pmc(kernel, P, B, pairs=True):
    """The newest committed PMC profile of (kernel, members per GPU, B) measured on the machine code the library
    holds now for that kernel instantiation (its kernel_isa_sha256; profiles without one: the decode sources'
    hash); (None, reason) when there is none (stale counters are never reported)."""
    import glob
    key = PMC_KEYS.get(kernel)
    if key is None:
        return None, None
    files = sorted(glob.glob(os.path.join(REPO, 'profiles', 'r*_pmc_%s_p%d_b%d.json' % (key, P, B))), reverse=True)
    if key == 'steps' and not pairs:     # the exact-lse instantiation's profile (measured on the trained-like theta)
        files += sorted(glob.glob(os.path.join(REPO, 'profiles', 'r*_pmc_steps-trained_p%d_b%d.json' % (P, B))),
                        reverse=True)
    if not files:
        return None, None
    symbol = PMC_SYMBOLS.get((key, pairs if key != 'sampled' else False))
    sha = kernel_source_sha256()
    for f in files:
        with open(f) as fh:
            rec = json.load(fh)
        if rec.get('kernel_isa_sha256'):
            ok = rec.get('kernel_symbol') == symbol and library_kernel_sha(symbol) == rec['kernel_isa_sha256']
        else:
            ok = rec.get('source_sha256') == sha
        if ok:
            rec['file'] = os.path.relpath(f, REPO)
            return rec, None
    reason = ('%s measured %s (machine code %s / source %s); the library holds %s: counters not reported (re-run the '
              'PMC passes)' % (os.path.relpath(files[0], REPO), rec.get('kernel_symbol'),
                               str(rec.get('kernel_isa_sha256'))[:12], str(rec.get('source_sha256'))[:12],
                               str(library_kernel_sha(symbol) if symbol else None)[:12]))
    print('bench.py: STALE PMC PROFILE: ' + reason, file=sys.stderr, flush=True)
    return None, reason


def cpu_baseline(args, B, P):
    """The reference CPU path (torch-CPU restatement, oracle/ref_worker.py) on this box's host cores:
    one single-threaded worker process per core -- the reference's cpu_count() - 2 workers (main.py:105),
    capped by the CPUs this job may use -- at least one member each, then the master leg (ranks, fp32
    weighted sum of the P noise vectors, Adam) at the full population P."""
    from oracle import ref_worker
    import nicnes.synthetic as S
    import torch
    dims = S.Dims()
    theta = S.init_theta(dims, 0)
    fc = S.fc_feats(B, dims.F, 1234, args.bu)
    m = ref_worker.FCModelRef()
    torch.nn.utils.vector_to_parameters(torch.from_numpy(theta), m.parameters())
    with torch.no_grad():
        base, _ = m.sample(torch.from_numpy(fc))
    gts, df, ref_len_raw = S.build_references(base.numpy(), dims.vocab_size, 4321, 5, 4096, dims.T)
    node = os.cpu_count() or 1
    usable = ref_worker.usable_cpus()
    cores = args.cpu_cores or max(1, min(node - 2, usable))
    table = S.noise_table(1 << 24, 123)
    rng = np.random.default_rng(0)
    n_members = cores * args.cpu_members_per_core
    offs = 64 * rng.integers(0, (table.size - dims.D) // 64, max(n_members, P))
    deltas = [np.float32(args.sigma) * table[o: o + dims.D] for o in offs[:n_members]]
    rate, fits, secs = ref_worker.time_members(theta, fc, gts, df, ref_len_raw, deltas, cores)
    fit_P = np.resize(fits, (P, 2))          # the master's input: P fitness pairs (values recycled)
    t_master, _ = ref_worker.time_master(fit_P, table, offs[:P], args.sigma, theta)
    t_iter = P / rate + t_master
    per_core = 1.0 / float(secs.mean())
    return {'value': round(P / t_iter, 4), 'unit': 'members/s', 'cores': cores, 'kind': 'port',
            'sample': '%d members (2 rollouts of %d rows = %d unique images x5, 18+18 steps, pure-Python CIDEr-D) '
                      'on %d single-threaded worker processes (reference rule cpu_count()-2 = %d, capped by the '
                      '%d CPUs this job may use); then the master leg at P = %d (ranks, fp32 weighted sum of the '
                      'P noise vectors, fp64 Adam): %.2f s. Iteration = P / worker rate + master leg.'
                      % (n_members, 5 * B, B, cores, node - 2, usable, P, t_master),
            'worker_members_per_s': round(rate, 4), 'master_leg_s': round(t_master, 3),
            'mean_s_per_member_per_core': round(float(secs.mean()), 3),
            'node_cpus': node,
            'node_projection_members_per_s': round(P / (P / (per_core * max(node - 2, 1)) + t_master), 4),
            'node_projection_note': 'the reference rule cpu_count()-2 on every host CPU at the measured per-core '
                                    'rate (linear, an upper bound for the reference)'}


def resolve_world(gpus, env):
    """(world, launched_here): the rank count this run uses. `gpus` is --gpus (None: not given).
    Under a launcher (WORLD_SIZE set) --gpus must name the same count; without one, --gpus N > 1 means
    this process starts the N ranks itself (launched_here True). Raises SystemExit(2) on a mismatch."""
    ws = env.get('WORLD_SIZE')
    if ws is not None:
        world = int(ws)
        if gpus is not None and gpus != world:
            print('bench.py: --gpus %d but WORLD_SIZE=%d: refusing to report a %d-rank run as %d GPUs'
                  % (gpus, world, world, gpus), file=sys.stderr, flush=True)
            raise SystemExit(2)
        return world, False
    n = 1 if gpus is None else int(gpus)
    if n < 1:
        raise SystemExit(2)
    return n, n > 1


def rank_environments(n, port, base):
    """The environment of each of the n rank processes, as torch.distributed.run sets it on one node."""
    out = []
    for r in range(n):
        env = dict(base)
        env.update({'RANK': str(r), 'LOCAL_RANK': str(r), 'WORLD_SIZE': str(n), 'LOCAL_WORLD_SIZE': str(n),
                    'GROUP_RANK': '0', 'MASTER_ADDR': '127.0.0.1', 'MASTER_PORT': str(port),
                    'HSA_ENABLE_IPC_MODE_LEGACY': base.get('HSA_ENABLE_IPC_MODE_LEGACY', '0')})
        out.append(env)
    return out


def free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


VISIBLE_DEVICE_VARS = ('ROCR_VISIBLE_DEVICES', 'HIP_VISIBLE_DEVICES', 'CUDA_VISIBLE_DEVICES')


def usable_gpu_count(env, topology='/sys/class/kfd/kfd/topology/nodes', dri='/dev/dri'):
    """GPUs the rank processes could use, counted WITHOUT any HIP / HSA call (the launcher must not
    initialise the GPU runtime: it only starts fresh rank processes). A GPU is a KFD topology node with
    SIMDs whose DRM render node this process can open (a cgroup that hides a GPU makes the open fail);
    a *_VISIBLE_DEVICES list caps the count. None when the topology cannot be read."""
    try:
        names = os.listdir(topology)
    except OSError:
        return None
    n = 0
    for name in sorted(names):
        props = {}
        try:
            with open(os.path.join(topology, name, 'properties')) as f:
                for line in f:
                    parts = line.split()
                    if len(parts) == 2:
                        props[parts[0]] = parts[1]
        except OSError:
            continue
        if int(props.get('simd_count', '0')) <= 0:
            continue                               # a CPU node
        minor = props.get('drm_render_minor')
        if minor is None:
            continue
        try:
            fd = os.open(os.path.join(dri, 'renderD%s' % minor), os.O_RDWR | os.O_CLOEXEC)
            os.close(fd)
        except OSError:
            continue
        n += 1
    for var in VISIBLE_DEVICE_VARS:
        val = env.get(var)
        if val is not None:
            n = min(n, len([v for v in val.split(',') if v.strip()]))
    return n


def launch_ranks(n, argv, grace=30.0):
    """Start n fresh rank processes running this script with `argv` (this process never touches the
    GPU: devices are counted from sysfs, usable_gpu_count), wait for all of them, and return the exit
    status: 0, or the first failing rank's (a rank killed by a signal counts as 1). When one rank fails
    the others are terminated. Status 2, before any rank starts, when fewer than n GPUs are usable or
    they cannot be counted."""
    shared = os.environ.get('NICNES_BENCH_SHARE_GPU') == '1'
    if not shared:
        have = usable_gpu_count(os.environ, os.environ.get('NICNES_BENCH_KFD_TOPOLOGY',
                                                           '/sys/class/kfd/kfd/topology/nodes'),
                                os.environ.get('NICNES_BENCH_DRI', '/dev/dri'))
        if have is None:
            print('bench.py: --gpus %d: cannot read the KFD topology to count GPUs' % n, file=sys.stderr, flush=True)
            return 2
        if have < n:
            print('bench.py: --gpus %d but %d GPUs are visible' % (n, have), file=sys.stderr, flush=True)
            return 2
    port = free_port()
    # rank 0's JSON line is the only stdout; everything else the ranks print (gloo / RCCL banners,
    # rank > 0) goes to stderr
    procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env,
                              stdout=subprocess.PIPE if r == 0 else sys.stderr.fileno(), text=r == 0)
             for r, env in enumerate(rank_environments(n, port, os.environ))]

    def forward(pipe):
        for line in pipe:
            (sys.stdout if line.startswith('{') else sys.stderr).write(line)
            (sys.stdout if line.startswith('{') else sys.stderr).flush()
    import threading
    fw = threading.Thread(target=forward, args=(procs[0].stdout,), daemon=True)
    fw.start()
    rc, alive, t_fail = 0, list(procs), None
    while alive:
        for p in list(alive):
            r = p.poll()
            if r is None:
                continue
            alive.remove(p)
            if r != 0 and rc == 0:
                rc = r if r > 0 else 1
                t_fail = time.time()
                for q in alive:
                    q.terminate()
        if alive and t_fail is not None and time.time() - t_fail > grace:
            for q in alive:
                q.kill()
        time.sleep(0.1)
    fw.join(timeout=10)
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=None, help='GPUs (= ranks); without a launcher this process '
                    'starts them (default: WORLD_SIZE, or 1)')
    ap.add_argument('--comm', choices=['torch', 'engine'], default='torch', help="the exchange's binding: "
                    "torch.distributed (RCCL as the 'nccl' backend) or the engine's own RCCL communicator "
                    "(nicnes_comm_init; its id shared over a gloo group)")
    ap.add_argument('--steps', type=int, default=5)
    ap.add_argument('--warmup', type=int, default=1)
    ap.add_argument('--preset', choices=sorted(PRESETS), default='metric', help='BASELINE.json config')
    ap.add_argument('--population', type=int, default=0, help='total population P, split over the N GPUs '
                    '(strong scaling; default: the preset\'s, 512 for the metric)')
    ap.add_argument('--pop-per-gpu', type=int, default=0, help='weak scaling instead: members per GPU (P = N x this)')
    ap.add_argument('--batch', type=int, default=0, help='unique images per batch (default: the preset\'s, 128)')
    ap.add_argument('--theta-gain', type=float, default=1.0, help='weight init gain (1: the reference xavier init; '
                    '4 with --bias-std 0.1: peaked, trained-like logits)')
    ap.add_argument('--bias-std', type=float, default=0.0)
    ap.add_argument('--batches', type=int, default=1, help='distinct batches per iteration (single_batch: false, '
                    'member i on batch i mod N)')
    ap.add_argument('--sigma', type=float, default=0.01)
    ap.add_argument('--noise-len', type=int, default=1 << 27)
    ap.add_argument('--bu', action='store_true', help="'bu' features: ReLU(N(0,1)) fc (configs[4]; implied by "
                    "--preset configs4)")
    ap.add_argument('--fitness', default='greedy', help="policy_options.fitness: greedy (mscoco_nes.json), "
                    "greedy_logprob / greedy_expprob / greedy_linprob / greedy_avgprob, or the sampled sample / "
                    "self_critical / sc_loss (every one of the batch's 5 rows per image decoded: the rows the "
                    "reference samples independently)")
    ap.add_argument('--mutation', default='', choices=['', 'SM-G-SUM', 'SM-PROPORTIONAL'],
                    help="model_options.safe_mutations (mscoco_nes.json: '', underflow 0.1): the per-task mutation "
                    "vector is recomputed from each iteration's theta on the host (nicnes.mutations) inside the "
                    "timed step, as reference workers do per task")
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--decode-split', type=int, default=0, help='force S logit workgroups per member (0 = auto)')
    ap.add_argument('--decode-rows', type=int, default=0, help='force 4 (128-row) or 2 (64-row) slabs (0 = auto)')
    ap.add_argument('--cpu-cores', type=int, default=0, help='worker processes (0: cpu_count()-2 capped by the usable CPUs)')
    ap.add_argument('--cpu-members-per-core', type=int, default=1)
    args = ap.parse_args()

    world, launch_here = resolve_world(args.gpus, os.environ)
    if launch_here:
        raise SystemExit(launch_ranks(world, sys.argv[1:]))
    rank = int(os.environ.get('RANK', '0'))
    local_rank = int(os.environ.get('LOCAL_RANK', '0'))
    P_pre, B_pre, bu_pre, cfg_text = PRESETS[args.preset]
    B = args.batch or B_pre
    args.bu = args.bu or bu_pre
    if args.pop_per_gpu:                     # weak scaling: a fixed share per GPU
        P_local, scaling = args.pop_per_gpu, 'weak'
        P = P_local * world
    else:                                    # strong scaling: a fixed population split over the GPUs
        P, scaling = args.population or P_pre, 'strong'
        if P % world:
            raise SystemExit('population %d does not split evenly over %d GPUs' % (P, world))
        P_local = P // world
    if os.environ.get('NICNES_BENCH_DRY_RANKS') == '1':
        # test hook (tests/test_bench_launcher.py): report the rank environment and the member range this rank
        # would evaluate (PopulationRunner's m0 = rank x P / N), then stop before any GPU work
        rec = {k: os.environ.get(k) for k in ('RANK', 'LOCAL_RANK', 'WORLD_SIZE', 'MASTER_ADDR', 'MASTER_PORT')}
        rec.update(members=[rank * P_local, (rank + 1) * P_local], population=P, batch=B, bu=bool(args.bu),
                   scaling=scaling)
        print(json.dumps(rec), flush=True)
        fail = os.environ.get('NICNES_BENCH_DRY_FAIL_RANK')
        if fail is not None and fail == os.environ.get('RANK'):
            raise SystemExit(3)
        return

    # CPU leg first, before this process touches the GPU (its pool forks)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args, B, P)

    import torch
    import torch.distributed as dist
    import nicnes
    import nicnes.synthetic as S
    from nicnes.population import PopulationRunner

    # rehearsal knobs for a one-GPU box (never set by the driver): every rank on cuda:0 over gloo
    backend = os.environ.get('NICNES_BENCH_BACKEND', 'nccl')
    share_gpu = os.environ.get('NICNES_BENCH_SHARE_GPU') == '1'
    dev = 0 if share_gpu else local_rank
    torch.cuda.set_device(dev)
    group = None
    if world > 1:
        if args.comm == 'engine':
            backend = 'gloo'                 # the bootstrap group: the data plane is the engine's communicator
        if backend == 'nccl':
            dist.init_process_group('nccl', device_id=torch.device('cuda', dev))
        else:
            dist.init_process_group(backend)
        if dist.get_world_size() != world or dist.get_rank() != rank:
            raise SystemExit('torch.distributed formed %d ranks (rank %d), expected %d (rank %d)'
                             % (dist.get_world_size(), dist.get_rank(), world, rank))
    # host tensors for the bench's own barrier / max-reduce on a gloo group, device tensors on RCCL
    red_dev = 'cuda' if (world > 1 and backend == 'nccl') else 'cpu'
    sampled = args.fitness in ('sample', 'self_critical', 'sc_loss')
    spi = 5 if sampled else 1               # sampled modes decode the reference's seq_per_img copies of each image
    eng = nicnes.Engine(max_batch=B, max_members=P_local, noise_len=args.noise_len, noise_seed=0, device=dev)
    wl = S.setup_engine_workload(eng, B=B, fc_seed=1235 if args.bu else 1234, bu=args.bu, batches=args.batches,
                                 theta_gain=args.theta_gain, bias_std=args.bias_std)
    eng.set_fitness_mode(args.fitness)
    if sampled:
        eng.set_rows_per_image(spi)          # each image's 5 copies decoded, each with its own draws
    eng.set_decode_split(args.decode_split, args.decode_rows)
    if share_gpu and world > 1:
        # ranks time-sharing one GPU (rehearsal only): the coop decode assumes the whole device
        eng.set_decode_coop(0)
    comm = None
    if world > 1 and args.comm == 'engine':
        uid = [nicnes.Engine.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        eng.comm_init(world, rank, uid[0])
        comm = 'engine'
    runner = PopulationRunner(eng, P, args.sigma, l2coeff=1e-7, stepsize=1e-3, rank=rank, world_size=world,
                              group=group, comm=comm)
    mut_s = []
    if args.mutation:
        # SM-G-SUM: Sensitivity.calc_sensitivity of the task's theta on its batch (safe_mutations.py:34-117),
        # per iteration; SM-PROPORTIONAL: |theta'| (nets.py:108-112)
        from types import SimpleNamespace
        from nicnes.mutations import Mutator
        spec = SimpleNamespace(model_options=SimpleNamespace(safe_mutations=args.mutation, safe_mutation_underflow=0.1,
                                                             safe_mutation_vector=''), batch_size=B)
        mutator = Mutator(spec, eng)
        fc_rows = wl['fc'][:B]

        def prepare(it_):
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ev0.record()
            mutator.prepare(it_, lambda: eng.theta()[1], fc_rows)   # SM-G-SUM: enqueued on the engine's stream
            ev1.record()
            mut_s.append((ev0, ev1))
    else:
        def prepare(it_):
            pass
    it = 1
    for _ in range(args.warmup):
        prepare(it)
        runner.step(it, sync=False, n_batches=args.batches)
        it += 1
    eng.set_timing(True)
    dec_ms, phases = [], []
    # per timed step: events on the engine's stream (torch's current stream) between the iteration's
    # three parts -- evaluate (decode + CIDEr-D), the fitness exchange, update (ranks, noise sum, its
    # all-reduce, Adam); runner.step issues exactly these calls
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    mut_s.clear()
    for k in range(args.steps):
        prepare(it)                                            # host sensitivity (waits for the last theta)
        e = evs[k]
        e[0].record()
        runner.evaluate(it, args.batches)                      # enqueue only (a batch map is one small copy)
        e[1].record()
        runner.exchange_fitness()
        e[2].record()
        runner.update(it, sync=False)
        e[3].record()
        it += 1
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    ratio = eng.last_ratio()
    # decode timing of the last timed step (HIP events recorded between its launches)
    dec_ms.append(eng.kernel_times()[0])
    phases.append(eng.decode_phase_times())
    part_ms = [float(np.mean([e[j].elapsed_time(e[j + 1]) for e in evs])) for j in range(3)]
    mine = [rank, runner.m0, runner.m0 + runner.local, dev, dt * 1e3 / args.steps] + part_ms
    ranks = [mine]
    comm_seen = {'binding': 'none (one rank)' if world == 1 else
                 ('engine RCCL communicator (nicnes_comm_init)' if comm == 'engine' else
                  'torch.distributed %s' % backend),
                 'world_size': dist.get_world_size() if world > 1 else 1}
    if comm == 'engine':
        comm_seen['rccl_comm_count'], comm_seen['rccl_rank'] = eng.comm_count()
    if world > 1:
        t = torch.tensor([dt], device=red_dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        row = torch.tensor(mine, device=red_dev, dtype=torch.float64)
        rows = [torch.zeros_like(row) for _ in range(world)]
        dist.all_gather(rows, row)
        ranks = [r.cpu().tolist() for r in rows]
        if comm == 'engine':
            n_seen = torch.tensor([comm_seen['rccl_comm_count']], device=red_dev, dtype=torch.float64)
            dist.all_reduce(n_seen, op=dist.ReduceOp.MIN)
            comm_seen['rccl_comm_count_min_over_ranks'] = int(n_seen.item())
    value = P * args.steps / dt
    mut_ms = float(np.mean([a.elapsed_time(b) for a, b in mut_s])) if mut_s else 0.0
    dec_s = float(np.mean(dec_ms)) / 1e3
    flops = decode_flops_per_member(B) * P_local
    # dominant kernel: the fused steps kernel (logits + token + next LSTM cell for every step t = -1..T,
    # one launch per evaluate) or, on the split path (members x slabs below the CU count), the logit kernel
    # (T launches); per-launch figures are the evaluate's totals / launches (what rocprofv3 --stats
    # averages over the same launches)
    ph = phases[-1]
    G, nslabs, S_split = eng.decode_shape(B, P_local)
    path = eng.decode_path(B, P_local)
    if sampled:
        # the sampled decode of the 5 B rows: the steps kernel, whose logit loop also stores each step's logits and
        # per-stage sums of p in its workgroup's slot; the pick scans the stage sums and walks one stage's logits
        # (one launch); the self-critical modes' greedy decode of the B images runs before it (in ms_per_step,
        # not here). Bytes: the noise rows + the stored logits written (their read-back is one stage per row).
        rows = B * spi
        G, nslabs, S_split, path = 4, (rows + 127) // 128, 1, 'fused (sampled pick)'
        kname, n_step = 'nicnes_decode_steps_kernel<sample>', 1
        step_ms = float(np.mean([q['step_ms'] for q in phases]))
        flops = decode_flops_per_member(rows) * P_local
        step_flop = step_flops_per_member(rows) * P_local
        # per workgroup and logit step: every 64-row stage's logits (64 KiB), its lanes' stage sums (8 KiB) and 8 KiB per 8 stages
        # written to the slot; the pick's reads (the stage sums up to the crossing stage, then one stage's
        # logits per row) are not counted
        nst = (9488 + 63) // 64
        slog_bytes = 16 * nslabs * (nst * 73728 + (nst + 7) // 8 * 8192)   # + the 8-stage block records
        alg_bytes = (step_noise_bytes_per_member(rows) + slog_bytes) * P_local
    elif not ph['step_launches'] and not ph['logit_launches']:
        # two-stream decode (NICNES_DECODE_STREAMS=2): the halves' launches overlap, so the whole decode
        # is the measured unit
        kname, n_step = 'decode (img + step/logit/cell kernels, 2 streams)', 1
        step_ms = float(np.mean(dec_ms))
        step_flop = flops
        alg_bytes = step_noise_bytes_per_member(B) * P_local
    elif ph['step_launches']:
        # fused path: every step of a workgroup in one launch (nicnes_decode_steps_kernel), or one launch
        # per step t = -1..T (nicnes_decode_step_kernel, DECODE_PROF timing builds); coop path: the split
        # shape's every step in one launch (nicnes_decode_coop_kernel, S workgroups per member slab)
        if path == 'coop':
            kname = 'nicnes_decode_coop_kernel<%d>' % S_split
        elif G == 2:                                 # 64-row slabs: nicnes_decode_steps2_kernel
            kname = 'nicnes_decode_steps2_kernel'
        else:
            kname = 'nicnes_decode_steps_kernel' if ph['step_launches'] == 1 else 'nicnes_decode_step_kernel'
            if args.mutation and G == 4 and ph['step_launches'] == 1:
                # a mutated member's embedding rows' delta' formed in the decode: its own kernel (no committed PMC
                # profile: the line reports traffic null rather than the plain kernel's counters)
                kname = 'nicnes_decode_steps_mut_kernel'
        n_step = ph['step_launches']
        step_ms = float(np.mean([q['step_ms'] for q in phases])) / n_step
        step_flop = step_flops_per_member(B) * P_local / n_step
        alg_bytes = step_noise_bytes_per_member(B) * P_local / n_step
    else:
        kname, n_step = 'nicnes_decode_logit_kernel<%d>' % G, ph['logit_launches']
        step_ms = float(np.mean([q['logit_ms'] for q in phases])) / n_step
        step_flop = logit_flops_per_member(B) * P_local / n_step
        alg_bytes = logit_noise_bytes_per_member() * P_local      # every member's logit noise, once per launch
    achieved = step_flop / (step_ms / 1e3) / 1e12
    # counter figures of the same kernel and workload from the committed rocprofv3 PMC profile
    # (a profile-derived constant: PMC passes cannot run inside the timed bench process)
    # (the instantiation the last timed decode ran: the greedy-only bounded-lse one, or the exact one -- log-probs
    # written, NICNES_BOUNDED_LSE=0, or the engine's adaptive policy on a peaked theta)
    pairs_run = args.fitness == 'greedy' and eng.last_decode_bounded()
    pmc, pmc_stale = load_pmc(kname, P_local, B, pairs_run)
    traffic = pmc['derived'].get('hbm_bytes_per_launch') if pmc else None
    hbm_peak_bytes = HBM_PEAK_GBS * 1e9 * step_ms / 1e3
    iter_bytes = iteration_algorithmic_bytes(B, P_local)
    out = {
        'metric': METRIC, 'value': round(value, 3), 'unit': 'members/s', 'n_gpus': world, 'steps': args.steps,
        'warmup': args.warmup, 'ms_per_step': round(dt / args.steps * 1e3, 3), 'higher_is_better': True,
        'scaling': scaling, 'vs_baseline': None, 'dtype': 'fp32',
        'data': 'synthetic (seeded fc features, xavier-init fc_caption theta, substituted refs, 2^27 noise table)',
        'config': {'baseline_config': args.preset if not (args.population or args.pop_per_gpu or args.batch)
                   else 'custom (%s preset overridden)' % args.preset,
                   'baseline_config_text': cfg_text,
                   'workload': 'mscoco_nes.json fc_caption, pop=%d antithetic (%d/GPU, %s scaling), batch_size=%d unique '
                               'images, sigma %.3g, full iteration (decode+CIDEr-D+ranks+noise sum+Adam)'
                               % (P, P_local, scaling, B, args.sigma) + (", 'bu' fc features" if args.bu else '')
                               + (', fitness %s' % args.fitness if args.fitness != 'greedy' else '')
                               + (' (%d rows per rollout: 5 sampled per image)' % (B * spi) if sampled else '')
                               + (', theta gain %g bias std %g (not the reference init)' % (args.theta_gain, args.bias_std)
                                  if (args.theta_gain != 1.0 or args.bias_std) else '')
                               + (', %d batches per iteration (single_batch false: member i on batch i mod %d)'
                                  % (args.batches, args.batches) if args.batches > 1 else '')
                               + (', safe_mutations %s' % args.mutation if args.mutation else ''),
                   'population': P, 'members_per_gpu': P_local, 'batch_size': B, 'batches_per_iteration': args.batches,
                   'seq_length': 16,
                   'vocab_size': 9487,
                   'parallelism': ('none (one GPU, no collective)' if world == 1 else
                                   'population-sharded x%d, %s all-gather of fitness + all-reduce of the noise sum'
                                   % (world, 'RCCL' if (backend == 'nccl' or comm == 'engine') else backend)),
                   'collective': comm_seen,
                   'shared_gpu_rehearsal': bool(share_gpu and world > 1)},
        'ranks': [{'rank': int(r[0]), 'members': [int(r[1]), int(r[2])], 'device': int(r[3]),
                   'ms_per_step': round(r[4], 3), 'evaluate_ms': round(r[5], 3), 'exchange_ms': round(r[6], 3),
                   'update_ms': round(r[7], 3)} for r in ranks],
        'roofline': {'bound': 'mfma', 'kernel': kname, 'achieved': round(achieved, 3),
                     'peak': FP32_MFMA_PEAK_TFLOPS, 'unit': 'TFLOP/s',
                     'frac': round(achieved / FP32_MFMA_PEAK_TFLOPS, 4), 'traffic': traffic,
                     'kernel_ms_per_launch': round(step_ms, 4), 'launches_per_step': n_step,
                     'algorithmic_flop_per_launch': step_flop,
                     'algorithmic_bytes_per_launch': alg_bytes,
                     'traffic_over_algorithmic': (round(traffic / alg_bytes, 3) if traffic else None),
                     'traffic_source': pmc['file'] if pmc else None,
                     'traffic_kernel_symbol': pmc.get('kernel_symbol') if pmc else None,
                     'traffic_stale': pmc_stale,
                     'hbm_frac': round(alg_bytes / hbm_peak_bytes, 4),
                     'hbm_frac_counters': round(traffic / hbm_peak_bytes, 4) if traffic else None,
                     'mfma_busy': round(pmc['derived']['mfma_busy'], 4) if pmc and 'mfma_busy' in pmc['derived'] else None,
                     'valu_insts_per_mfma': (round(pmc['derived']['valu_insts_per_mfma'], 3)
                                             if pmc and 'valu_insts_per_mfma' in pmc['derived'] else None),
                     'iteration_hbm_frac': round(iter_bytes * args.steps / dt / 1e9 / HBM_PEAK_GBS, 4),
                     'iteration_algorithmic_bytes': iter_bytes,
                     'decode': {'ms_per_step': round(dec_s * 1e3, 3), 'algorithmic_flop': flops,
                                'tflops': round(flops / dec_s / 1e12, 3),
                                'frac': round(flops / dec_s / 1e12 / FP32_MFMA_PEAK_TFLOPS, 4),
                                'img_ms': round(float(np.mean([q['img_ms'] for q in phases])), 3),
                                'cell_only_ms': round(float(np.mean([q['cell_only_ms'] for q in phases])), 3),
                                'step_ms': round(ph['step_ms'], 3), 'logit_ms': round(ph['logit_ms'], 3),
                                'cell_ms': round(ph['cell_ms'], 3),
                                'shape': {'row_groups': G, 'slabs': nslabs, 'logit_split': S_split},
                                'path': path}},
        'cpu_baseline': cpu,
        'decodes_per_s': round(2 * value, 3),        # one decode = one sign's rollout of the batch
        'tie_fallbacks': eng.stats()['tie_fallbacks'],
        'sample_stage_fallbacks': eng.stats()['sample_stage_fallbacks'] if sampled else None,
        'mutation': ({'mode': args.mutation, 'vector_ms_per_iteration': round(mut_ms, 3),
                      'vector_share_of_iteration': round(mut_ms / (dt / args.steps * 1e3), 4),
                      'note': 'the per-task mutation vector, timed with events on the engine stream: SM-G-SUM '
                              '= nicnes_sum_sensitivity (the sigma 0 token decode + 95 batched backward passes of '
                              'a 5-step decode, safe_mutations.py:93-117), SM-PROPORTIONAL = |theta| formed on the device '
                              '(nicnes_set_mutation_proportional; the host mean only when theta has exact zeros)'}
                     if args.mutation else None),
        'update_ratio': ratio,
    }
    if rank == 0:
        print(json.dumps(out), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
