"""Real-data readers (nicnes.data) against the behaviour of the reference's
captioning DataLoader (src/captioning/dataloader.py:35-315) on a small dataset written here, and
the CiderD df-table formats. CPU only."""
import collections
import json
import os
import pickle

import numpy as np
import pytest

from nicnes import data as Dt
from nicnes.config import NotSupported
from nicnes.nes import unique_batch


@pytest.fixture()
def dataset(tmp_path):
    rng = np.random.default_rng(0)
    splits = ['train', 'val', 'test', 'restval', 'train', 'train', 'restval', 'val']
    images = [{'id': 100 + i, 'split': sp, 'file_path': 'img%d.jpg' % i} for i, sp in enumerate(splits)]
    info = {'ix_to_word': {str(i): 'w%d' % i for i in range(1, 30)}, 'images': images}
    with open(tmp_path / 'cocotalk.json', 'w') as f:
        json.dump(info, f)
    os.makedirs(tmp_path / 'fc')
    for im in images:
        np.save(tmp_path / 'fc' / ('%d.npy' % im['id']), rng.standard_normal(16).astype(np.float32))
    ncap = [5, 6, 2, 5, 7, 5, 1, 5]                      # images 2 and 6 have fewer than seq_per_img
    start = np.cumsum([0] + ncap[:-1]) + 1               # 1-based, inclusive (dataloader.py:129-130)
    labels = rng.integers(1, 30, (sum(ncap), 16))
    labels[:, 10:] = 0
    Dt.LabelStore(labels, start, start + np.array(ncap) - 1).save_npz(str(tmp_path / 'labels.npz'))
    return tmp_path, images, labels, start, ncap


def _loader(tmp_path, **kw):
    return Dt.CocoFcDataLoader(str(tmp_path / 'cocotalk.json'), str(tmp_path / 'fc'), str(tmp_path / 'labels.npz'),
                               batch_size=3, **kw)


def test_splits_vocab_and_restval(dataset):
    tmp_path, images, _, _, _ = dataset
    L = _loader(tmp_path)
    assert L.vocab_size == 29 and L.get_seq_length() == 16
    assert sorted(L.split_ix['train']) == [0, 3, 4, 5, 6]          # restval joins train (train_only 0)
    assert L.split_ix['val'] == [1, 7] and L.split_ix['test'] == [2]
    assert sorted(_loader(tmp_path, train_only=1).split_ix['train']) == [0, 4, 5]


def test_get_batch_matches_reference_layout(dataset):
    tmp_path, images, labels, start, ncap = dataset
    L = _loader(tmp_path)
    b = L.get_batch('train')
    assert b['fc_feats'].shape == (15, 16) and b['fc_feats'].dtype == np.float32
    assert b['labels'].shape == (15, 18) and (b['labels'][:, 0] == 0).all() and (b['labels'][:, -1] == 0).all()
    for i, inf in enumerate(b['infos']):
        ix = inf['ix']
        assert inf['id'] == images[ix]['id']
        fc = np.load(tmp_path / 'fc' / ('%d.npy' % inf['id']))
        assert all(np.array_equal(b['fc_feats'][5 * i + q], fc) for q in range(5))
        rows = labels[start[ix] - 1: start[ix] - 1 + ncap[ix]]
        assert np.array_equal(b['gts'][i], rows)                   # every label row of the image
        mine = b['labels'][5 * i: 5 * i + 5, 1:17]
        assert all(any(np.array_equal(r, g) for g in rows) for r in mine)
        if ncap[ix] >= 5:                                        # a contiguous window of 5 rows
            first = [j for j in range(ncap[ix]) if np.array_equal(rows[j], mine[0])][0]
            assert np.array_equal(mine, rows[first:first + 5])
    fc_u, gts = unique_batch(b)
    assert fc_u.shape == (3, 16) and len(gts) == 3


def test_walk_wraps_and_reshuffles(dataset):
    tmp_path = dataset[0]
    L = _loader(tmp_path, seed=3)
    seen = []
    for _ in range(2):
        b = L.get_batch('val', batch_size=1)
        seen.append(b['infos'][0]['ix'])
    assert sorted(seen) == [1, 7] and b['bounds']['wrapped'] and b['bounds']['it_pos_now'] == 0
    epoch = [L.get_batch('train', batch_size=1)['infos'][0]['ix'] for _ in range(5)]
    assert sorted(epoch) == [0, 3, 4, 5, 6]
    a = _loader(tmp_path, seed=9).get_batch('train', batch_size=5)
    c = _loader(tmp_path, seed=9).get_batch('train', batch_size=5)
    assert [x['ix'] for x in a['infos']] == [x['ix'] for x in c['infos']]     # seeded: replayable


def test_h5_labels_need_h5py(tmp_path):
    pytest.importorskip('numpy')
    try:
        import h5py  # noqa: F401
        pytest.skip('h5py present')
    except ImportError:
        pass
    with pytest.raises(NotSupported):
        Dt.LabelStore.load(str(tmp_path / 'cocotalk_label.h5'))


def _df():
    return {('1',): 3.0, ('1', '2'): 2.0, ('4', '5', '6'): 1.0, ('7', '8', '9', '10'): 1.0}


@pytest.mark.parametrize('protocol', [0, 2, 4])
def test_df_pickle_restricted_load(tmp_path, protocol):
    """The upstream CiderD df pickle: {'document_frequency': defaultdict(float), 'ref_len': n}."""
    p = tmp_path / 'coco-train-idxs.p'
    dd = collections.defaultdict(float, _df())
    with open(p, 'wb') as f:
        pickle.dump({'document_frequency': dd, 'ref_len': 4096.0}, f, protocol=protocol)
    df, ref_len = Dt.load_df_table(str(p))
    assert df == _df() and ref_len == 4096.0


def test_df_pickle_refuses_code(tmp_path):
    class Evil:
        def __reduce__(self):
            return (os.system, ('true',))
    p = tmp_path / 'evil.p'
    with open(p, 'wb') as f:
        pickle.dump({'document_frequency': {}, 'ref_len': Evil()}, f)
    with pytest.raises(pickle.UnpicklingError):
        Dt.load_df_table(str(p))


@pytest.mark.parametrize('ext', ['json', 'npz'])
def test_df_portable_roundtrip(tmp_path, ext):
    p = str(tmp_path / ('df.' + ext))
    Dt.save_df_table(p, _df(), 4096)
    df, ref_len = Dt.load_df_table(p)
    assert df == _df() and ref_len == 4096.0


def test_loader_feeds_master_loop(dataset, tmp_path):
    """A real-data batch stream drives the master loop (oracle engine, tiny dims) end to end."""
    import itertools
    from nicnes import config as C
    from nicnes import master as M
    from oracle import oracle as O
    from tests.cpu_engine import OracleEngine
    dpath = dataset[0]
    L = _loader(dpath)
    dims = O.Dims(vocab_size=29, E=32, R=32, F=16)
    theta = O.make_theta(dims, 2, 4.0, 0.1)
    df, ref_len = {('1',): 2.0, ('2', '3'): 1.0}, 8.0
    table = O.noise_table(1 << 16, 123)
    e = OracleEngine(dims, theta, np.zeros((3, 16), np.float32), [], df, ref_len, table)
    exp = {'algorithm': 'nic_nes', 'dataset': 'mscoco', 'nb_offspring': 4,
           'config': {'noise_stdev': 0.05, 'batch_size': 3, 'l2coeff': 1e-3, 'snapshot_freq': 0},
           'policy_options': {'net': 'fc_caption', 'fitness': 'greedy'},
           'optimizer_options': {'type': 'adam', 'args': {'stepsize': 0.01}}}
    m = M.EngineMaster(C.ExperimentSpec(exp, vocab_size=29), e, log_dir=str(tmp_path / 'log'))
    m.run(itertools.islice(Dt.batches(L), 2), max_iterations=2)
    assert m.opt.t == 2 and len(m.stats) == 2
