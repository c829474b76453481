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
