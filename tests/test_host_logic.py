"""Host-side logic of the engine package (no GPU): synthetic workload generators and their
agreement with the oracle's definitions."""
import numpy as np

import nicnes.synthetic as S
from oracle import oracle as O


def test_init_theta_matches_oracle_definition():
    for dims_args in ((63, 32, 32, 64), (9487, 128, 128, 2048)):
        d = S.Dims(*dims_args)
        od = O.Dims(*dims_args)
        assert d.D == od.D
        assert np.array_equal(S.init_theta(d, 3, 2.0, 0.1), O.make_theta(od, 3, 2.0, 0.1))


def test_noise_table_is_the_oracle_table():
    assert np.array_equal(S.noise_table(4096, 123), O.noise_table(4096, 123))


def test_substituted_refs_format():
    rng = np.random.Generator(np.random.PCG64(0))
    rows = S.substituted_refs(np.arange(1, 17), 9487, rng, 5, 16)
    assert rows.shape == (5, 16) and rows.dtype == np.int32
    for r in rows:
        nz = np.nonzero(r == 0)[0]
        L = nz[0] + 1 if len(nz) else 16
        assert 8 <= L <= 16
        assert np.all(r[:L - 1] > 0) and np.all(r[L:] == 0)


def test_build_references_df_counts_documents():
    base = np.tile(np.arange(1, 17), (4, 1))
    gts, df, n = S.build_references(base, 50, seed=1, n_refs=5, df_sets=32)
    assert n == 32 and len(gts) == 4
    assert max(df.values()) <= 32 and min(df.values()) >= 1
    # every n-gram of a batch ref appears in the df table
    w = [int(t) for t in gts[0][0] if True]
    assert (w[0],) in df


def test_fc_features_bu_nonnegative():
    assert (S.fc_feats(4, 2048, 1235, bu=True) >= 0).all()
    assert (S.fc_feats(4, 2048, 1234) < 0).any()


def _binade_half_ulp(a):
    """decode_kernel.hip binade_half_ulp: 2^(E - 24) for a in [2^E, 2^(E+1)), 0 for tiny a."""
    ex = int(np.float32(a).view(np.uint32)) >> 23
    return float(np.uint32((ex - 24) << 23).view(np.float32)) if ex > 24 else 0.0


def test_pair_bound_tie_window_rule():
    """The rule the greedy-only decode uses when lse is only bounded (decode_kernel.hip tie_window /
    win_state): for every lse in [lo, hi], e <= hu_in decides 'in', e > hu_out decides 'out', where the
    exact test is fp32(-e - lse) == -lse (torch's log_softmax tie, nets.py:208-209); e == half an ulp
    is the one case that depends on lse's last bit (taken as in)."""
    rng = np.random.default_rng(5)
    f32 = np.float32
    for _ in range(3000):
        base = f32(rng.uniform(0.01, 9.3))
        lo, hi = f32(base - f32(2e-3)), f32(base + f32(0.69314718 + 2e-3))
        hu_in = _binade_half_ulp(lo) if lo > 0 else 0.0
        hu_out = _binade_half_ulp(hi)
        # true lse anywhere in the interval, candidates at multiples of a logit ulp around the half-ulps
        lse = f32(rng.uniform(float(lo), float(hi)))
        u = float(np.spacing(f32(rng.uniform(0.5, 12.0))))
        for e in {f32(k * u) for k in range(0, 40)} | {f32(hu_in), f32(hu_out), f32(2 * hu_out)}:
            exact_in = (f32(-e) - lse) == -lse
            if e == 0 or e <= hu_in:
                if e != _binade_half_ulp(lse) or e == 0:
                    assert exact_in, (lse, e, hu_in)
            elif e > hu_out:
                assert not exact_in, (lse, e, hu_out)
