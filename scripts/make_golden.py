"""Generate tests/golden/ fixtures from the REFERENCE implementation (runs in the build container only).

The reference tree (/root/reference, read-only) is imported here to produce input/output vectors;
nothing from it is copied into the repo and nothing in tests/, bench.py or the engine reads it at
run time. Re-run with:  PYTHONDONTWRITEBYTECODE=1 python scripts/make_golden.py

Fixtures (all .npz, loadable with allow_pickle=False):
  decode_tiny_{xavier,wc}.npz     FCModel._sample (src/captioning/nets.py:183-245) on tiny dims,
                                  theta stored in full; reference seq/logprobs + top-2 margins
  decode_full_{xavier,wc}.npz     full fc_caption dims (V=9487, E=R=128, F=2048); theta and fc are
                                  regenerated from the stored seeds (oracle.make_theta / numpy PCG64),
                                  plus two table-perturbed members (theta+delta, theta-delta)
  perturb_semantics.npz           PolicyNet.evolve (src/algorithm/nets.py:83-119): new params ==
                                  fp32(theta + delta), and worker's theta - delta (nic_nes_worker.py:151)
  adam.npz                        Adam.update (src/algorithm/nic_nes/optimizers.py:15-22,78-83) driven
                                  like NESMaster.run_master (nic_nes_master.py:126-133), 3 steps
  ranks.npz                       compute_centered_ranks docstring known answer (nic_nes_master.py:187-189)
  sgd.npz                         SGD.update (optimizers.py:38-47) driven like run_master, 3 steps
  adam_globalg64.npz              Adam.update(globalg) called directly with an fp64 globalg from the
                                  first step (the fp64 (1 - b) * g' branch while theta is still fp32)
  decode_bench_xavier.npz         the bench workload itself (BASELINE.json configs[2] inputs: xavier theta seed
                                  0, fc PCG64(1234) [128, 2048], the 2^27 table PCG64(123), noise seed 0,
                                  iteration 1): FCModel._sample on the reference's 5x-duplicated 640 rows
                                  (dataloader.py:175) for base theta and 16 table-perturbed members x 2 signs
                                  (8 of them below 64, so the pop=64 split path is pinned on 2,048 rows);
                                  tokens of each image's first copy, per-step top-2 margins, logprobs, and
                                  whether the 5 copies of every image decoded identically
  decode_bench_b64.npz            the same at mscoco_nes.json's own batch_size 64 (experiments/mscoco_nes.json:7):
                                  the first 64 images (320 duplicated rows), the 64-row slab path of the engine
  decode_rank_slices.npz          the per-GPU slices of the 8-GPU configs: configs[3] rank 7 (members 1792-2047
                                  of pop 2048) on the bench inputs, configs[4] rank 7 (members 448-511, plus
                                  members of rank 0) on bottom-up ReLU(N(0,1)) features (fc seed 1235)
  master_ranks_grad.npz          NESMaster.compute_centered_ranks / gradient_estimate
                                  (nic_nes_master.py:170-221) imported with placeholder redis/torchvision
                                  modules: P = 512 tie-free fitness and a tied one, and the fp32 gradient
                                  of 512 table-noise vectors on 4096 sampled coordinates
  wire_reference.npz              the reference's wire bytes: dist.serialize (src/dist.py:25-26, pickle
                                  protocol -1) of an NESTask (nic_nes_master.py:27-28) as the master declares
                                  it (a batch dict of numpy arrays / lists / dicts), of (task_id, NESResult) as
                                  a worker pushes it (nic_nes_worker.py:156-161, dist.py:199-201), and of an
                                  experiment dict (dist.py:73-76)
  mutations.npz                   PolicyNet.evolve with safe / proportional mutations (src/algorithm/nets.py:83-119):
                                  the raw normal_ draw, the returned noise (raw / sensitivity, raw * |theta'|)
                                  for SM-G-SUM with a set sensitivity and for SM-PROPORTIONAL; and the SM-G-SUM
                                  sensitivity itself, Sensitivity.calc_sensitivity (safe_mutations.py:34-117)
                                  on a tiny FCModel through forward_for_sensitivity (captioning/nets.py:22-70)
  decode_sample.npz               FCModel._sample(greedy=False) (nets.py:210-231) with the global numpy RNG
                                  seeded: tokens, seq_logprobs and the uniforms RandomState.choice drew
                                  (replayed and checked step by step), tiny and full dims
  fitness_criteria.npz            the greedy_* fitness criteria and sc_loss's LogFitnessCriterion
                                  (src/captioning/fitness.py:12-132, chosen
                                  by Fitness.get_criterium, src/captioning/policies.py:50-61) on seeded
                                  logprobs / sequences / per-row CIDEr rewards, as CaptPolicy.rollout
                                  calls them (policies.py:119-123)
Pass fixture names to regenerate a subset: python scripts/make_golden.py sgd adam_globalg64
"""
import json
import os
import sys
from collections import namedtuple

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, '/root/reference/src')

from oracle import oracle as O  # noqa: E402

import captioning.nets as ref_nets  # noqa: E402  (reference module)

OUT = os.path.join(REPO, 'tests', 'golden')
os.makedirs(OUT, exist_ok=True)
torch.set_num_threads(1)          # the reference pins one thread per worker (src/main.py:8-11)
torch.set_grad_enabled(False)

Opt = namedtuple('Opt', ['vocab_size', 'input_encoding_size', 'rnn_size', 'fc_feat_size', 'vbn', 'vbn_e',
                         'vbn_affine', 'layer_n', 'layer_n_affine', 'safe_mutations',
                         'safe_mutation_underflow', 'safe_mutation_vector'])


def ref_model(d):
    opt = Opt(d.vocab_size, d.E, d.R, d.F, False, False, False, False, False, '', 0.1, '')
    return ref_nets.FCModel(options=opt)


def load_theta(model, theta32):
    torch.nn.utils.vector_to_parameters(torch.from_numpy(np.ascontiguousarray(theta32)), model.parameters())


def ref_decode(model, fc):
    """Reference greedy decode + per-step top-2 log-prob margin (replayed with the model's own
    modules in the same op order as FCModel._sample; the replayed tokens are asserted equal)."""
    fct = torch.from_numpy(fc)
    seq, slp = model._sample(fct, greedy=True)
    B = fc.shape[0]
    state = model.init_hidden(B)
    margins = np.full((B, model.seq_length), np.inf, np.float32)
    xt = model.img_embed(fct)
    _, state = model.core(xt, state)
    it = fct.new_zeros(B, dtype=torch.long)
    unfinished = None
    for t in range(1, model.seq_length + 1):
        xt = model.embed(it)
        out, state = model.core(xt, state)
        lp = torch.nn.functional.log_softmax(model.logit(out), dim=1)
        top = lp.topk(2, 1).values
        margins[:, t - 1] = (top[:, 0] - top[:, 1]).numpy()
        _, it = torch.max(lp, 1)
        unfinished = (it > 0) if t == 1 else unfinished * (it > 0)
        it = it * unfinished.type_as(it)
        assert torch.equal(it, seq[:, t - 1]), 'replay diverged from _sample'
        if unfinished.sum() == 0:
            break
    return seq.numpy().astype(np.int32), slp.numpy().astype(np.float32), margins


def decode_fixture(name, d, theta_seed, gain, bias_std, fc_seed, B, store_theta, members=()):
    model = ref_model(d)
    theta = O.make_theta(d, theta_seed, gain, bias_std)
    fc = np.random.Generator(np.random.PCG64(fc_seed)).standard_normal((B, d.F)).astype(np.float32)
    load_theta(model, theta)
    seq, slp, mar = ref_decode(model, fc)
    out = dict(dims=np.array([d.vocab_size, d.E, d.R, d.F, d.T], np.int64),
               theta_seed=np.int64(theta_seed), gain=np.float64(gain), bias_std=np.float64(bias_std),
               fc_seed=np.int64(fc_seed), B=np.int64(B), seq=seq, logprobs=slp, margins=mar)
    if store_theta:
        out['theta'] = theta
        out['fc'] = fc
    # table-perturbed members (theta +- fp32(sigma z)), the engine's noise contract
    if members:
        T, tseed, nseed, it, sigma = 1 << 23, 123, 7, 3, 0.01
        table = O.noise_table(T, tseed)
        out.update(noise_len=np.int64(T), table_seed=np.int64(tseed), noise_seed=np.int64(nseed),
                   iteration=np.int64(it), sigma=np.float64(sigma), members=np.array(members, np.int64))
        pseq, pmar = [], []
        for mbr in members:
            idx = O.noise_index(nseed, it, mbr, T, d.D)
            for sign in (+1, -1):
                load_theta(model, O.perturb(theta, table, idx, sigma, sign))
                s, _, m = ref_decode(model, fc)
                pseq.append(s)
                pmar.append(m)
        out['member_seq'] = np.stack(pseq)       # [members*2, B, T] order (m0+, m0-, m1+, ...)
        out['member_margins'] = np.stack(pmar)
    np.savez_compressed(os.path.join(OUT, name + '.npz'), **out)
    print(name, 'seq[0]', seq[0], 'min margin', float(mar.min()))


BENCH_MEMBERS = np.array(sorted(set(np.linspace(0, 511, 8).astype(np.int64).tolist())
                                | {8, 16, 24, 32, 40, 48, 63, 100}), np.int64)


def decode_bench_fixture(B=128, name='decode_bench_xavier'):
    d = O.Dims()
    model = ref_model(d)
    theta = O.make_theta(d, 0, 1.0, 0.0)               # = nicnes.synthetic.init_theta(Dims(), 0)
    T_LEN, TSEED, NSEED, IT, SIGMA = 1 << 27, 123, 0, 1, 0.01
    # the first B rows of the bench's PCG64(1234) [128, 2048] draw (numpy fills in C order)
    fc = np.random.Generator(np.random.PCG64(1234)).standard_normal((B, d.F)).astype(np.float32)
    fc5 = np.repeat(fc, 5, axis=0)                     # the reference decodes every image 5 times
    table = O.noise_table(T_LEN, TSEED)
    members = BENCH_MEMBERS
    seqs, mars, lps, dup = [], [], [], []

    def run(th):
        load_theta(model, th)
        s5, lp5, m5 = ref_decode(model, fc5)
        s5, lp5, m5 = s5.reshape(B, 5, -1), lp5.reshape(B, 5, -1), m5.reshape(B, 5, -1)
        dup.append(bool((s5 == s5[:, :1]).all()))
        seqs.append(s5[:, 0])
        mars.append(m5[:, 0])
        lps.append(lp5[:, 0])

    run(theta)                                         # base theta: the synthetic references' seed captions
    for mbr in members:
        idx = O.noise_index(NSEED, IT, int(mbr), T_LEN, d.D)
        for sign in (+1, -1):
            run(O.perturb(theta, table, idx, SIGMA, sign))
    np.savez_compressed(os.path.join(OUT, name + '.npz'), B=np.int64(B), noise_len=np.int64(T_LEN),
                        table_seed=np.int64(TSEED), noise_seed=np.int64(NSEED), iteration=np.int64(IT),
                        sigma=np.float64(SIGMA), members=members, seq=np.stack(seqs).astype(np.int16),
                        margins=np.stack(mars), logprobs=np.stack(lps), dup_consistent=np.array(dup))
    print(name, 'copies consistent', all(dup), 'min margin', float(np.stack(mars).min()))


def ref_sample(model, fc, seed):
    """FCModel._sample(greedy=False) (nets.py:210-231) with the global numpy RNG seeded, and the uniforms it
    drew: RandomState.choice(len, 1, p) takes one random_sample() per call, one call per row and step
    (rows in order) from t = 0 (the image step, whose pick is discarded) until every row has finished. The draws are replayed from the same seed and the decode
    is re-run step by step with the reference's own modules and that choice rule (cdf = cumsum(p / |p|_1) in
    fp64 / its last entry, searchsorted side='right'); the replayed tokens are asserted equal, which pins
    the draw order. Returns seq, seq_logprobs, u [B, T] (0 after the last step drawn) and the distance of
    each draw from the nearest cdf boundary of its pick (u_margin, inf where not drawn)."""
    fct = torch.from_numpy(fc)
    np.random.seed(seed)
    seq, slp = model._sample(fct, greedy=False)
    B, T = seq.shape
    np.random.seed(seed)
    # the loop samples at t = 0 too (the image step, nets.py:203-224; its pick is replaced by <bos>), so
    # B draws precede logit step 1's
    draws = np.random.random_sample(B * (T + 1)).reshape(T + 1, B)[1:]
    u = np.zeros((B, T), np.float64)
    margin = np.full((B, T), np.inf)
    state = model.init_hidden(B)
    _, state = model.core(model.img_embed(fct), state)
    it = fct.new_zeros(B, dtype=torch.long)
    unfinished = None
    for t in range(1, T + 1):
        out, state = model.core(model.embed(it), state)
        lp = torch.nn.functional.log_softmax(model.logit(out), dim=1)
        prob = torch.exp(lp).numpy()
        pick = np.zeros(B, np.int64)
        for b in range(B):
            n_row = prob[b] / np.linalg.norm(prob[b], ord=1)
            cdf = n_row.astype(np.float64).cumsum()
            cdf /= cdf[-1]
            ub = draws[t - 1, b]
            k = int(cdf.searchsorted(ub, side='right'))
            pick[b] = k
            u[b, t - 1] = ub
            margin[b, t - 1] = min(abs(cdf[k] - ub), abs(ub - cdf[k - 1]) if k > 0 else np.inf)
        itn = torch.from_numpy(pick)
        unfinished = (itn > 0) if t == 1 else unfinished * (itn > 0)
        it = itn * unfinished.type_as(itn)
        assert torch.equal(it, seq[:, t - 1]), 'replayed draws diverged from _sample'
        if unfinished.sum() == 0:
            break
    return seq.numpy().astype(np.int32), slp.numpy().astype(np.float32), u, margin


def decode_sample_fixture():
    """decode_sample.npz: FCModel._sample(greedy=False) on tiny dims (stored theta, peaked and flat) and on
    the full fc_caption dims (xavier and peaked theta from their seeds, 40 rows), with the draws."""
    out = {}
    cases = [('tiny_wc', O.Dims(vocab_size=63, E=32, R=32, F=64), 2, 4.0, 0.1, 8, 11),
             ('tiny_xavier', O.Dims(vocab_size=63, E=32, R=32, F=64), 1, 1.0, 0.0, 8, 12),
             ('full_xavier', O.Dims(), 0, 1.0, 0.0, 40, 13),
             ('full_wc', O.Dims(), 0, 4.0, 0.1, 40, 14)]
    for name, d, tseed, gain, bstd, B, seed in cases:
        model = ref_model(d)
        theta = O.make_theta(d, tseed, gain, bstd)
        load_theta(model, theta)
        fc = np.random.Generator(np.random.PCG64(1234)).standard_normal((B, d.F)).astype(np.float32)
        seq, slp, u, mar = ref_sample(model, fc, seed)
        out.update({name + '_dims': np.array([d.vocab_size, d.E, d.R, d.F, d.T], np.int64),
                    name + '_theta_seed': np.int64(tseed), name + '_gain': np.float64(gain),
                    name + '_bias_std': np.float64(bstd), name + '_B': np.int64(B), name + '_seq': seq,
                    name + '_logprobs': slp, name + '_u': u, name + '_u_margin': mar})
        print(name, 'seq[0]', seq[0], 'min u margin', float(mar.min()))
    np.savez_compressed(os.path.join(OUT, 'decode_sample.npz'), **out)


def decode_bench_b64_fixture():
    decode_bench_fixture(64, 'decode_bench_b64')


# the last rank's slice of each multi-GPU BASELINE config (member ranges as bench.py --gpus 8 shards them)
SLICE_C3 = np.array([1792, 1793, 1830, 1871, 1920, 1966, 2001, 2047], np.int64)       # configs[3]: P=2048, rank 7
SLICE_C4 = np.array([0, 7, 33, 63, 448, 449, 470, 490, 511], np.int64)               # configs[4]: P=512, rank 7 (+ rank 0)


def decode_rank_slices_fixture():
    """decode_rank_slices.npz: FCModel._sample on the per-GPU slices of the two 8-GPU BASELINE configs.
    c3 = configs[3] (pop = 2048 over 8 GPUs: rank 7 evaluates members 1792..2047) on the bench inputs (xavier
    theta seed 0, fc PCG64(1234) N(0,1), B = 128, 5x-duplicated rows); c4 = configs[4] (bottom-up features:
    ReLU of PCG64(1235) N(0,1), nicnes.synthetic.fc_feats(bu=True); pop = 512 over 8 GPUs: rank 7 evaluates
    members 448..511, plus members of rank 0's slice). Same table / noise seed / iteration / sigma as
    decode_bench_xavier. Per case: seq [1 + 2 * members, B, T] (base theta first, then m+, m- per member) of
    each image's first copy, margins, logprobs, dup_consistent."""
    d = O.Dims()
    model = ref_model(d)
    theta = O.make_theta(d, 0, 1.0, 0.0)
    T_LEN, TSEED, NSEED, IT, SIGMA, B = 1 << 27, 123, 0, 1, 0.01, 128
    table = O.noise_table(T_LEN, TSEED)
    out = dict(B=np.int64(B), noise_len=np.int64(T_LEN), table_seed=np.int64(TSEED), noise_seed=np.int64(NSEED),
               iteration=np.int64(IT), sigma=np.float64(SIGMA))
    for case, fc_seed, bu, members in (('c3', 1234, False, SLICE_C3), ('c4', 1235, True, SLICE_C4)):
        fc = np.random.Generator(np.random.PCG64(fc_seed)).standard_normal((B, d.F)).astype(np.float32)
        if bu:
            fc = np.maximum(fc, 0.0).astype(np.float32)
        fc5 = np.repeat(fc, 5, axis=0)
        seqs, mars, lps, dup = [], [], [], []
        for k in range(-1, len(members)):
            for sign in ((0,) if k < 0 else (+1, -1)):
                th = theta if k < 0 else O.perturb(theta, table, O.noise_index(NSEED, IT, int(members[k]), T_LEN,
                                                                                d.D), SIGMA, sign)
                load_theta(model, th)
                s5, lp5, m5 = ref_decode(model, fc5)
                s5, lp5, m5 = s5.reshape(B, 5, -1), lp5.reshape(B, 5, -1), m5.reshape(B, 5, -1)
                dup.append(bool((s5 == s5[:, :1]).all()))
                seqs.append(s5[:, 0])
                mars.append(m5[:, 0])
                lps.append(lp5[:, 0])
        out.update({case + '_fc_seed': np.int64(fc_seed), case + '_bu': np.bool_(bu), case + '_members': members,
                    case + '_seq': np.stack(seqs).astype(np.int16), case + '_margins': np.stack(mars),
                    case + '_logprobs': np.stack(lps), case + '_dup_consistent': np.array(dup)})
        print('rank slice', case, 'copies consistent', all(dup), 'min margin', float(np.stack(mars).min()))
    np.savez_compressed(os.path.join(OUT, 'decode_rank_slices.npz'), **out)


class _Placeholder(__import__('types').ModuleType):
    """stands in for a module the reference imports but this path never uses (redis, torchvision)"""
    def __getattr__(self, k):
        if k.startswith('__'):
            raise AttributeError(k)
        return _Placeholder(self.__name__ + '.' + k)


def master_ranks_grad_fixture():
    np.float = float
    for name in ('redis', 'torchvision'):
        try:
            __import__(name)
        except ImportError:
            sys.modules[name] = _Placeholder(name)
    from algorithm.nic_nes.nic_nes_master import NESMaster   # reference module
    master = NESMaster.__new__(NESMaster)                     # the rank/sum methods use no state
    rng = np.random.Generator(np.random.PCG64(55))
    P = 512
    fit = rng.standard_normal((P, 2)) * 10.0 + 50.0          # tie-free
    fit_ties = np.round(rng.random((P, 2)) * 40) / 4.0       # many ties
    cr = master.compute_centered_ranks(fit)
    cr_ties = master.compute_centered_ranks(fit_ties)
    d = O.Dims()
    T_LEN, NSEED, IT, SIGMA = 1 << 27, 0, 1, 0.01
    table = O.noise_table(T_LEN, 123)
    idx = np.array([O.noise_index(NSEED, IT, i, T_LEN, d.D) for i in range(P)], np.int64)
    J = np.sort(np.random.Generator(np.random.PCG64(3)).choice(d.D, 4096, replace=False)).astype(np.int64)
    vecs = np.float32(SIGMA) * table[idx[:, None] + J[None, :]]                  # delta_i[J], fp32
    g = master.gradient_estimate(fit, vecs)
    np.savez_compressed(os.path.join(OUT, 'master_ranks_grad.npz'), fit=fit, cr=cr, fit_ties=fit_ties,
                        cr_ties=cr_ties, noise_len=np.int64(T_LEN), noise_seed=np.int64(NSEED),
                        iteration=np.int64(IT), sigma=np.float64(SIGMA), idx=idx, J=J, grad=np.asarray(g))
    print('master: grad dtype', np.asarray(g).dtype, 'max|g|', float(np.abs(g).max()))


def wire_fixture():
    for name in ('redis', 'torchvision'):
        try:
            __import__(name)
        except ImportError:
            sys.modules[name] = _Placeholder(name)
    np.float = float
    from algorithm.nic_nes.nic_nes_master import NESTask, NESResult   # reference wire types
    from dist import serialize                                       # reference codec
    rng = np.random.Generator(np.random.PCG64(21))
    B, T = 3, 16
    fc = rng.standard_normal((B * 5, 32)).astype(np.float32)
    gts = [rng.integers(0, 50, (int(n), T)).astype(np.uint32) for n in (5, 6, 5)]
    labels = np.zeros((B * 5, T + 2), dtype='int')
    labels[:, 1:T + 1] = rng.integers(0, 50, (B * 5, T))
    batch = {'fc_feats': fc, 'att_feats': np.zeros((B * 5, 1, 1), np.float32), 'labels': labels,
             'masks': (labels > 0).astype(np.float32), 'att_masks': None, 'gts': gts,
             'bounds': {'it_pos_now': 3, 'it_max': 113287, 'wrapped': False},
             'infos': [{'ix': 7 * i, 'id': 1000 + i, 'file_path': 'train2014/COCO_%d.jpg' % i} for i in range(B)]}
    task = NESTask(current='logs/nic_nes_mscoco_fc_caption_1/models/current/0_current_params.pth', batch_data=batch,
                   noise_stdev=0.01, log_dir='logs/nic_nes_mscoco_fc_caption_1', ref_batch=None, batch_size=B)
    D = 1000
    noise = (np.float32(0.01) * rng.standard_normal(D).astype(np.float32))
    fitness = np.stack((71.25, 64.5))
    result = NESResult(worker_id=3, evolve_noise=noise, fitness=fitness, mem_usage=123456789)
    eval_result = NESResult(worker_id=4, eval_score=55.5, mem_usage=1234)
    with open('/root/reference/experiments/mscoco_nes.json') as f:
        exp = json.load(f)
    np.savez_compressed(os.path.join(OUT, 'wire_reference.npz'),
                        task_bytes=np.frombuffer(serialize(task), np.uint8),
                        result_bytes=np.frombuffer(serialize((7, result)), np.uint8),
                        eval_bytes=np.frombuffer(serialize((7, eval_result)), np.uint8),
                        exp_bytes=np.frombuffer(serialize(exp), np.uint8),
                        noise=noise, fitness=fitness, fc=fc, labels=labels,
                        gts_flat=np.concatenate(gts), gts_rows=np.array([len(g) for g in gts]))
    print('wire: task %d B, result %d B' % (len(serialize(task)), len(serialize((7, result)))))


def mutations_fixture():
    import tempfile
    d = O.Dims(vocab_size=63, E=32, R=32, F=64)
    B = 4
    theta = O.make_theta(d, 5, 4.0, 0.0)                  # zero biases: SM-PROPORTIONAL's mean replacement
    fc = np.random.Generator(np.random.PCG64(66)).standard_normal((B, d.F)).astype(np.float32)

    def model(mode, underflow=0.1):
        opt = Opt(d.vocab_size, d.E, d.R, d.F, False, False, False, False, False, mode, underflow, '')
        m = ref_nets.FCModel(options=opt)
        load_theta(m, theta)
        return m
    # SM-G-SUM sensitivity on the batch (5 duplicated rows per image, as the loader gives)
    m = model('SM-G-SUM', 0.1)
    with tempfile.TemporaryDirectory() as tmp:
        m.calc_sensitivity(0, 0, {'fc_feats': np.repeat(fc, 5, axis=0)}, B, tmp)
    sens = m.get_sensitivity_vector().numpy().astype(np.float32)
    # evolve with that sensitivity
    torch.manual_seed(11)
    raw = torch.empty(d.D).normal_(mean=0.0, std=0.01).numpy()
    torch.manual_seed(11)
    delta_safe = m.evolve(0.01)
    # SM-PROPORTIONAL
    mp_ = model('SM-PROPORTIONAL')
    torch.manual_seed(11)
    delta_prop = mp_.evolve(0.01)
    np.savez_compressed(os.path.join(OUT, 'mutations.npz'), theta=theta, fc=fc, dims=np.array([d.vocab_size, d.E, d.R, d.F]),
                        underflow=np.float64(0.1), sensitivity=sens, raw=raw, delta_safe=delta_safe,
                        delta_prop=delta_prop)
    print('mutations: sens min %.3g max %.3g' % (sens.min(), sens.max()))


def perturb_fixture():
    d = O.Dims(vocab_size=63, E=32, R=32, F=64)
    model = ref_model(d)
    theta = O.make_theta(d, 5)
    load_theta(model, theta)
    torch.manual_seed(11)
    delta = model.evolve(0.01)                                     # reference PolicyNet.evolve
    plus = torch.nn.utils.parameters_to_vector(model.parameters()).numpy().copy()
    minus = (torch.from_numpy(theta) - torch.from_numpy(delta)).numpy()   # nic_nes_worker.py:151
    np.savez_compressed(os.path.join(OUT, 'perturb_semantics.npz'), theta=theta, delta=delta, plus=plus,
                        minus=minus)
    print('perturb: plus==theta+delta', bool(np.array_equal(plus, theta + delta)))


def adam_fixture():
    np.float = float        # numpy>=1.24 removed the alias optimizers.py:75-76 uses
    from algorithm.nic_nes.optimizers import Adam   # reference module
    rng = np.random.Generator(np.random.PCG64(99))
    D = 1000
    theta32 = rng.standard_normal(D).astype(np.float32)
    grads = rng.standard_normal((3, D)).astype(np.float32) * np.float32(0.05)
    l2coeff, stepsize = 1e-3, 1e-2
    opt = Adam(theta32.copy(), stepsize)
    theta = theta32.copy()
    thetas, ratios, ms, vs = [], [], [], []
    for k in range(3):
        reg = l2coeff * theta                    # nic_nes_master.py:311 restated (fp32 first step)
        ratio, theta = opt.update(-grads[k] + reg)
        thetas.append(np.asarray(theta, np.float64))
        ratios.append(ratio)
        ms.append(opt.m.copy())
        vs.append(opt.v.copy())
    np.savez_compressed(os.path.join(OUT, 'adam.npz'), theta0=theta32, grads=grads, l2coeff=np.float64(l2coeff),
                        stepsize=np.float64(stepsize), thetas=np.stack(thetas), ratios=np.array(ratios),
                        ms=np.stack(ms), vs=np.stack(vs))
    print('adam ok, ratio', ratios)


def sgd_fixture():
    np.float = float
    from algorithm.nic_nes.optimizers import SGD    # reference module
    rng = np.random.Generator(np.random.PCG64(98))
    D = 1000
    theta32 = rng.standard_normal(D).astype(np.float32)
    grads = rng.standard_normal((3, D)).astype(np.float32) * np.float32(0.05)
    l2coeff, stepsize, momentum = 1e-3, 1e-2, 0.9
    opt = SGD(theta32.copy(), stepsize, momentum)
    theta = theta32.copy()
    thetas, ratios, vs = [], [], []
    for k in range(3):
        reg = l2coeff * theta
        ratio, theta = opt.update(-grads[k] + reg)
        thetas.append(np.asarray(theta, np.float64))
        ratios.append(ratio)
        vs.append(opt.v.copy())
    np.savez_compressed(os.path.join(OUT, 'sgd.npz'), theta0=theta32, grads=grads, l2coeff=np.float64(l2coeff),
                        stepsize=np.float64(stepsize), momentum=np.float64(momentum), thetas=np.stack(thetas),
                        ratios=np.array(ratios), vs=np.stack(vs))
    print('sgd ok, ratio', ratios)


def adam_globalg64_fixture():
    np.float = float
    from algorithm.nic_nes.optimizers import Adam   # reference module
    rng = np.random.Generator(np.random.PCG64(97))
    D = 1000
    theta32 = rng.standard_normal(D).astype(np.float32)
    globalgs = rng.standard_normal((2, D)) * 0.05          # fp64
    opt = Adam(theta32.copy(), 1e-2)
    thetas = []
    for k in range(2):
        _, theta = opt.update(globalgs[k])
        thetas.append(np.asarray(theta, np.float64))
    np.savez_compressed(os.path.join(OUT, 'adam_globalg64.npz'), theta0=theta32, globalgs=globalgs,
                        stepsize=np.float64(1e-2), thetas=np.stack(thetas), m=opt.m.copy(), v=opt.v.copy())
    print('adam_globalg64 ok')


def ranks_fixture():
    # docstring known answer, /root/reference/src/algorithm/nic_nes/nic_nes_master.py:187-189
    x = np.array([[101, 200], [2, 100]], np.float64)
    y = np.array([[0.16666667, 0.5], [-0.5, -0.16666667]])
    np.savez_compressed(os.path.join(OUT, 'ranks.npz'), x=x, y=y)


def fitness_criteria_fixture():
    import captioning.fitness as ref_fit  # noqa: E402  (reference module)
    crits = {'greedy_logprob': ref_fit.AltLogFitnessCriterion, 'greedy_expprob': ref_fit.ExpFitnessCriterion,
             'greedy_linprob': ref_fit.LinFitnessCriterion, 'greedy_avgprob': ref_fit.AvgLogFitnessCriterion,
             'sc_loss': ref_fit.LogFitnessCriterion}
    rng = np.random.Generator(np.random.PCG64(77))
    cases = {}
    for case, (N, T) in enumerate([(8, 16), (40, 16), (5, 16)]):
        seq = rng.integers(1, 50, (N, T)).astype(np.int64)
        for i in range(N):                      # rows end at a random step (some never, one at t = 0)
            end = 0 if i == 0 else int(rng.integers(1, T + 4))
            if end < T:
                seq[i, end:] = 0
        lp = (-rng.exponential(1.5, (N, T))).astype(np.float32)
        scores = rng.uniform(0, 3, N).astype(np.float64)
        if case == 2:
            scores[:] = 0.0
        if case == 1:                           # self-critical rewards (sample - greedy) take either sign
            scores -= 1.5
        cases['seq_%d' % case], cases['lp_%d' % case], cases['scores_%d' % case] = seq, lp, scores
        reward = np.repeat(scores[:, None], T, 1)          # compute_ciders, policies.py:191
        for name, cls in crits.items():
            out = cls()(torch.from_numpy(lp), torch.from_numpy(seq), torch.from_numpy(reward).float())
            cases['%s_%d' % (name, case)] = np.array(float(out.item()))
    np.savez_compressed(os.path.join(OUT, 'fitness_criteria.npz'), **cases)


def all_fixtures():
    tiny = O.Dims(vocab_size=63, E=32, R=32, F=64)
    full = O.Dims()
    decode_fixture('decode_tiny_xavier', tiny, 1, 1.0, 0.0, 1234, 8, True)
    decode_fixture('decode_tiny_wc', tiny, 2, 4.0, 0.1, 1234, 8, True)
    decode_fixture('decode_full_xavier', full, 0, 1.0, 0.0, 1234, 16, False, members=(0, 1))
    decode_fixture('decode_full_wc', full, 0, 4.0, 0.1, 1234, 16, False, members=(0, 1))
    decode_sample_fixture()
    perturb_fixture()
    adam_fixture()
    ranks_fixture()
    sgd_fixture()
    adam_globalg64_fixture()
    fitness_criteria_fixture()
    decode_bench_fixture()
    decode_bench_b64_fixture()
    decode_rank_slices_fixture()
    master_ranks_grad_fixture()
    wire_fixture()
    mutations_fixture()


if __name__ == '__main__':
    if len(sys.argv) > 1:
        for name in sys.argv[1:]:
            globals()[name + '_fixture']()
    else:
        all_fixtures()
    with open(os.path.join(OUT, 'MANIFEST.json'), 'w') as f:
        json.dump({'generator': 'scripts/make_golden.py', 'reference': 'rubencart/NES-img-captioning @ /root/reference',
                   'torch': torch.__version__, 'numpy': np.__version__, 'threads': 1}, f, indent=1)
