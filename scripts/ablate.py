"""Decode-kernel ablation: time timing-only builds (make -C nes-img-captioning_amd ablate) in ONE
process on ONE GPU, interleaved rounds (cdna_hip_programming.md 5.4 rule 24). Dev tool."""
import glob
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'nes-img-captioning_amd'))
import nicnes  # noqa: E402
import nicnes.synthetic as S  # noqa: E402


def launch_spans(k, seq):
    """DECODE_PROF=1 build: per-launch span, workgroup durations, per-CU busy time, in-kernel clock."""
    raw = seq.reshape(-1, 4096).cpu().numpy().astype(np.int64) & 0xffffffff
    ts, cyc, hw = raw[:, :1024], raw[:, 1024:2048], raw[:, 2048:]
    launches = [('img', 80)] + [('step%d' % t, 2 * (t + 1)) for t in range(-1, 17)]
    t0 = ts[:, 80].min()
    rows = []
    for name, sl in launches:
        st = (ts[:, sl] - t0) % (1 << 32)
        en = (ts[:, sl + 1] - t0) % (1 << 32)
        dur = (en - st) / 100.0                               # us (100 MHz counter)
        ghz = np.median(((cyc[:, sl + 1] - cyc[:, sl]) % (1 << 32)) / np.maximum(dur, 1e-3) / 1e3)
        span = (en.max() - st.min()) / 100.0
        per_cu = {}
        for c_, d_ in zip(hw[:, sl], dur):
            per_cu[c_] = per_cu.get(c_, 0.0) + d_
        busy = np.array(list(per_cu.values()))
        rows.append((name, st.min() / 100.0, span, dur.mean(), dur.min(), dur.max(), len(per_cu),
                     busy.mean(), busy.max(), busy.mean() / span, ghz))
    print(k, 'launch: start_us span_us wg_mean wg_min wg_max n_cu cu_busy_mean cu_busy_max eff(mean busy/span) GHz')
    for r in sorted(rows, key=lambda r: r[1]):
        print('%-8s %9.1f %8.1f %8.1f %8.1f %8.1f %4d %8.1f %8.1f %6.3f %5.2f' % r)


def cell_stages(k, seq):
    """DECODE_PROF=1 build, step launches t = 1..15: median wave-0 time (us) of the logit loop, the token
    phase, and each cell stage m (marks 120 + 24 (t + 1) + {0: after the logit loop, 1: cell start,
    2 + m: after cell stage m})."""
    raw = seq.reshape(-1, 4096).cpu().numpy().astype(np.int64) & 0xffffffff
    ts = raw[:, :1024]
    rows = {'logit': [], 'token': [], 'cell': []}
    per_m = [[] for _ in range(20)]
    for t in range(1, 16):
        b = 120 + 24 * (t + 1)
        st = ts[:, 2 * (t + 1)]
        rows['logit'].append(np.median(((ts[:, b] - st) % (1 << 32)) / 100.0))
        rows['token'].append(np.median(((ts[:, b + 1] - ts[:, b]) % (1 << 32)) / 100.0))
        prev = ts[:, b + 1]
        for m in range(20):
            cur = ts[:, b + 2 + m]
            per_m[m].append(np.median(((cur - prev) % (1 << 32)) / 100.0))
            prev = cur
        rows['cell'].append(np.median(((ts[:, b + 21] - ts[:, b + 1]) % (1 << 32)) / 100.0))
    print(k, 'median over t=1..15 (us): logit %.1f token %.1f cell %.1f' % tuple(np.median(rows[x]) for x in
                                                                                ('logit', 'token', 'cell')))
    print(k, 'cell stage m (us):', ' '.join('%d:%.2f' % (m, np.median(v)) for m, v in enumerate(per_m)))
    if os.environ.get('FITNESS', '') in ('sample', 'self_critical', 'sc_loss'):   # the pick's marks 22, 23
        sp = {'to_l1': [], 'l1_to_l2': [], 'l2_to_cell': []}
        for t in range(1, 16):
            b = 120 + 24 * (t + 1)
            sp['to_l1'].append(np.median(((ts[:, b + 22] - ts[:, b]) % (1 << 32)) / 100.0))
            sp['l1_to_l2'].append(np.median(((ts[:, b + 23] - ts[:, b + 22]) % (1 << 32)) / 100.0))
            sp['l2_to_cell'].append(np.median(((ts[:, b + 1] - ts[:, b + 23]) % (1 << 32)) / 100.0))
        print(k, 'sampled token phase (us):', ' '.join('%s %.1f' % (n, np.median(v)) for n, v in sp.items()))


def split_spans(k, seq, S=4):
    """DECODE_PROF=1 build, split path (64 members, S = 4): per launch span, mean workgroup time and the gap
    to the previous launch's last workgroup; cell launches t = 1..15 split into merge / stage fill / 5 tiles."""
    raw = seq.reshape(-1, 1024).cpu().numpy().astype(np.int64) & 0xffffffff
    ts = raw[:, :256]
    launches = [('img', 250, 251), ('cell-1', 32, 43), ('cell0', 44, 55)]
    for t in range(1, 17):
        launches.append(('logit%d' % t, 2 * t - 2, 2 * t - 1))
        if t < 16:
            launches.append(('cell%d' % t, 32 + 12 * (t + 1), 32 + 12 * (t + 1) + 11))
    t0 = ts[:, 250].min()
    print(k, 'split launch: start_us span_us wg_mean wg_min wg_max gap_us')
    prev_end = None
    for name, a, b in launches:
        st = ((ts[:, a] - t0) % (1 << 32)) / 100.0
        en = ((ts[:, b] - t0) % (1 << 32)) / 100.0
        dur = en - st
        gap = st.min() - prev_end if prev_end is not None else 0.0
        print('%-8s %9.1f %8.1f %8.1f %8.1f %8.1f %7.1f' % (name, st.min(), en.max() - st.min(), dur.mean(),
                                                          dur.min(), dur.max(), gap))
        prev_end = en.max()
    sub = [[] for _ in range(4)]
    for t in range(1, 16):
        b = 32 + 12 * (t + 1)
        marks = [b, b + 8, b + 9, b + 10, b + 1]
        for i in range(4):
            sub[i].append(np.median(((ts[:, marks[i + 1]] - ts[:, marks[i]]) % (1 << 32)) / 100.0))
    print(k, 'merge split (us): entry->alive %.1f partials %.1f compute %.1f token+sync %.1f' % tuple(
        np.median(v) for v in sub))
    ph = [[] for _ in range(8)]
    for t in range(1, 16):
        b = 32 + 12 * (t + 1)
        marks = [b, b + 1, b + 2, b + 3, b + 4, b + 5, b + 6, b + 7, b + 11]
        for i in range(8):
            ph[i].append(np.median(((ts[:, marks[i + 1]] - ts[:, marks[i]]) % (1 << 32)) / 100.0))
    print(k, 'cell t=1..15 median (us): merge %.1f fill %.1f tiles %s end %.1f' % (
        np.median(ph[0]), np.median(ph[1]), ' '.join('%.1f' % np.median(v) for v in ph[2:7]), np.median(ph[7])))


def coop_spans(k, seq, S, pop):
    """DECODE_PROF=1 build, coop path (one launch, S workgroups per member slab): per step t = 1..15 the
    median over workgroups of the logit loop, the phase-A wait (partials), the merge + token, the cell,
    the phase-B wait (h'), and the read-back of h to the next step's start; then the logit loop per range q
    (the slowest range sets the pace of its group)."""
    raw = seq.reshape(-1, 1024).cpu().numpy().astype(np.int64) & 0xffffffff
    nwg = S * pop                                  # the launch's workgroups (one 128-row slab per member)
    ts = raw[:nwg, :256]
    names = ('logit', 'waitA', 'token', 'cell', 'waitB', 'to_next')
    ph = {n: [] for n in names}
    per_q = [[] for _ in range(S)]
    for t in range(1, 16):
        b = 8 * (t + 1)
        marks = [b, b + 1, b + 2, b + 3, b + 4, b + 5, b + 8]
        for i, n in enumerate(names):
            d = ((ts[:, marks[i + 1]] - ts[:, marks[i]]) % (1 << 32)) / 100.0
            ph[n].append(np.median(d))
        d = ((ts[:, b + 1] - ts[:, b]) % (1 << 32)) / 100.0
        for q in range(S):
            per_q[q].append(np.median(d[np.arange(nwg) % S == q]))
    tot = ((ts[:, 8 * 17 + 1] - ts[:, 8 * 2]) % (1 << 32)) / 100.0
    print(k, 'coop median per step t=1..15 (us):', ' '.join('%s %.2f' % (n, np.median(v)) for n, v in ph.items()))
    print(k, 'coop logit loop by range q (us):', ' '.join('q%d %.2f' % (q, np.median(v)) for q, v in enumerate(per_q)))
    print(k, 'coop steps 1..16 span per workgroup (us): median %.1f max %.1f' % (np.median(tot), tot.max()))


def main():
    pop = int(os.environ.get('POP', '512'))
    B = int(os.environ.get('BATCH', '128'))
    rounds = int(os.environ.get('ROUNDS', '3'))
    # ABLATE_DIR: where the variant libraries are (build/ is not shipped to the GPU box: copy them out)
    adir = os.environ.get('ABLATE_DIR', os.path.join(REPO, 'nes-img-captioning_amd', 'build', 'ablate'))
    libs = sorted(glob.glob(os.path.join(adir, 'libnicnes_*.so')))
    noise = torch.from_numpy(S.noise_table(1 << 27)).cuda()
    engines = {}
    only = [x for x in os.environ.get('ONLY', '').split(',') if x]
    if only:
        libs = [p for p in libs if os.path.basename(p)[len('libnicnes_'):-3] in only + ['base']]
    libs.sort(key=lambda p: not p.endswith('_base.so'))          # base first: it makes the refs
    wl = None
    for path in libs:
        name = os.path.basename(path)[len('libnicnes_'):-3]
        e = nicnes.Engine(max_batch=B, max_members=pop, noise_len=1 << 27, lib_path=path)
        if wl is None:
            wl = S.setup_engine_workload(e, B=B, noise=noise)
            keys, vals = nicnes.df_table_arrays(wl['df'])
        else:                                   # timing-only builds decode garbage: reuse base's refs
            e.set_noise_table(noise)
            e.set_theta(wl['theta32'])
            e.set_df_table(keys, vals, np.log(float(wl['ref_len_raw'])))
            e.set_batch(wl['fc'], wl['gts'])
        fit = os.environ.get('FITNESS', '')    # e.g. 'sample': the sampled kernel, 5 rows per image
        if fit:
            e.set_fitness_mode(fit)
            if fit in ('sample', 'self_critical', 'sc_loss'):
                e.set_rows_per_image(5)
        e.set_timing(True)
        engines[name] = e
    res = {k: [] for k in engines}
    phase = {k: [] for k in engines}
    for r in range(rounds):
        for k, e in engines.items():
            e.evaluate(r + 1, 0, pop, 0.01)
            res[k].append(e.kernel_times()[0])
            phase[k].append(e.decode_phase_times())
    ref = engines['base'].evaluate(99, 0, 8, 0.01, return_seq=True)
    for k in [x for x in os.environ.get('EXACT', '').split(',') if x]:   # variants that must match base
        if k in engines:
            got = engines[k].evaluate(99, 0, 8, 0.01, return_seq=True)
            print(k, 'tokens == base:', bool(torch.equal(got[1], ref[1])), 'fitness == base:',
                  bool(torch.equal(got[0], ref[0])))
    for k in [x for x in engines if x.startswith('prof')]:   # DECODE_PROF builds: per-WG launch spans
        torch.cuda.synchronize()
        time.sleep(0.05)
        e = engines[k]
        seqs = []
        gsum = torch.empty(e.D, dtype=torch.float32, device='cuda')
        for q in range(3):                      # bench-like iterations, nothing waits in between
            fit, seq = e.evaluate(50 + q, 0, pop, 0.01, return_seq=True)
            _, w = e.rank_weights(fit)
            e.grad_partial(50 + q, 0, pop, w, 0.01, out=gsum)
            e.adam_step(gsum, pop, 1e-7, 1e-6, sync=False)
            seqs.append(seq)
        for q, seq in enumerate(seqs):
            print('--- %s iteration %d of 3 (decode, CIDEr-D, ranks, noise sum, Adam), queued after a 50 ms idle'
                  % (k, q + 1))
            path = e.decode_path(B, pop)
            if path == 'coop':
                coop_spans(k, seq, e.decode_shape(B, pop)[2], pop)
            elif pop <= 64:
                split_spans(k, seq)
            else:
                launch_spans(k, seq)
                cell_stages(k, seq)
    base = np.median(res['base'])
    out = {k: {'median_ms': round(float(np.median(v)), 3), 'min_ms': round(float(np.min(v)), 3),
               'vs_base': round(float(np.median(v) / base), 3),
               'step_ms': round(float(np.median([ph['step_ms'] for ph in phase[k]])), 3),
               'cell_only_ms': round(float(np.median([ph['cell_only_ms'] for ph in phase[k]])), 3),
               'img_ms': round(float(np.median([ph['img_ms'] for ph in phase[k]])), 3),
               'tie_fallbacks': engines[k].stats()['tie_fallbacks']} for k, v in res.items()}
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main()
