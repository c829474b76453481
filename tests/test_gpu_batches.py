"""Per-member batches on the GPU (single_batch: false, nic_nes_worker.py:121-128): one launch
evaluates members on different batches (member i on batch member_batch[i]); every member's tokens
and CIDEr-D fitness equal the oracle's on its own batch, for the per-image-table and the
per-reference-scan scorers and for the fused and split decode paths."""
import numpy as np
import pytest

torch = pytest.importorskip('torch')

pytestmark = pytest.mark.gpu

from oracle import oracle as O          # noqa: E402
from oracle import cider_ref as CR      # noqa: E402

NOISE_LEN = 1 << 23
SIGMA = 0.01


@pytest.mark.parametrize('n_refs', [5, 10], ids=['image_tables', 'scan_over_8_refs'])
@pytest.mark.parametrize('shape', [(0, 0), (1, 4), (4, 2)], ids=['auto', 'fused', 'split_G2S4'])
def test_members_on_their_own_batches(n_refs, shape):
    import nicnes
    import nicnes.synthetic as S
    dims = O.Dims()
    theta = O.make_theta(dims, 3, 4.0, 0.1)
    G, B, P = 3, 20, 6
    rng = np.random.Generator(np.random.PCG64(202))
    fcs = [rng.standard_normal((B, dims.F)).astype(np.float32) for _ in range(G)]
    bases = [O.decode(dims, theta, f)[0] for f in fcs]
    gts_all, df, n = S.build_references(np.concatenate(bases), dims.vocab_size, seed=8, n_refs=n_refs, df_sets=256)
    gts = [gts_all[g * B:(g + 1) * B] for g in range(G)]
    table = O.noise_table(NOISE_LEN, 123)
    e = nicnes.Engine(max_batch=8, max_members=P, noise_len=NOISE_LEN, noise_seed=4)
    try:
        e.set_noise_table(table)
        keys, vals = nicnes.df_table_arrays(df)
        e.set_df_table(keys, vals, np.log(float(n)))
        e.set_theta(theta)
        e.set_batches(list(zip(fcs, gts)))                 # grows past max_batch=8 (20 rows, 60 images)
        e.set_decode_split(*shape)
        mb = [2, 0, 1, 1, 2, 0]
        fit, seq = e.evaluate(5, 0, P, SIGMA, return_seq=True, member_batch=mb)
        fit, seq = fit.cpu().numpy(), seq.cpu().numpy()
        scorer = CR.CiderDOracle(df, n)
        for k in range(P):
            idx = O.noise_index(4, 5, k, NOISE_LEN, dims.D)
            for s, sign in enumerate((+1, -1)):
                oseq, _, fr = O.decode(dims, O.perturb(theta, table, idx, SIGMA, sign), fcs[mb[k]])
                assert not fr.any() and np.array_equal(seq[k, s], oseq), (k, s)
                f_ref = CR.rollout_fitness(scorer, oseq, gts[mb[k]])[0]
                assert abs(fit[k, s] - f_ref) <= 1e-9 * max(1.0, f_ref), (k, s, fit[k, s], f_ref)
        with pytest.raises(nicnes.NicnesError):
            e.evaluate(5, 0, P, SIGMA)                      # several batches held: the map is required
        with pytest.raises(nicnes.NicnesError):
            e.evaluate(5, 0, 2, SIGMA, member_batch=[0, 3])  # batch 3 does not exist
    finally:
        e.close()
