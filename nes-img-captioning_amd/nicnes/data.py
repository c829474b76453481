"""Real-data readers for the engine's inputs: the captioning DataLoader's fc path
and the fixed document-frequency table of CIDEr-D.

Mirrors /root/reference/src/captioning/dataloader.py:
  DataLoader.__init__        :35-125   info json (ix_to_word, images + split), labels + pointers,
                                       split assignment (restval -> train when train_only == 0)
  DataLoader.get_captions    :127-146  seq_per_img label rows per image, subsampled with
                                       replacement when an image has fewer
  DataLoader.get_batch       :148-203  fc_feats repeated seq_per_img times, labels [B*spi, L+2],
                                       gts (every label row of the image), bounds, infos
  DataLoader.__getitem__     :209-243  fc feature of image ix = np.load(<fc_dir>/<id>.npy)
  BlobFetcher._get_next_minibatch_inds :300-315  sequential walk over the split, wrap + reshuffle
and the df file CiderD(df='coco-train-idxs') opens (captioning/policies.py:72; upstream cider:
pickle {'document_frequency': {n-gram tuple of word strings: count}, 'ref_len': #reference sets}).

Differences, on purpose:
  * labels come from the reference's cocotalk_label.h5 when h5py is importable; this image has no
    h5py, so the same three arrays are also read from an .npz ('labels', 'label_start_ix',
    'label_end_ix') -- `np.load(allow_pickle=False)`.
  * the df pickle is read by a restricted unpickler that builds only dicts, tuples, strings,
    numbers and collections.defaultdict(float); anything else in the file raises, nothing in it
    is executed. A JSON / npz export (`save_df_table`) is offered as the portable form.
  * the random generator is a seeded `random.Random` owned by the loader instead of the module-wide
    `random` state, so a master and its tests can replay a batch sequence.
"""
import collections
import io
import json
import os
import pickle
import random

import numpy as np

from .config import NotSupported


# ---------------------------------------------------------------- labels --------------------------
class LabelStore:
    """The three arrays of cocotalk_label.h5: labels [n_captions, L] int, label_start_ix /
    label_end_ix [n_images] (1-based, inclusive), dataloader.py:68-78."""

    def __init__(self, labels, label_start_ix, label_end_ix):
        self.labels = np.asarray(labels)
        self.label_start_ix = np.asarray(label_start_ix).astype(np.int64)
        self.label_end_ix = np.asarray(label_end_ix).astype(np.int64)
        if self.labels.ndim != 2 or self.label_start_ix.shape != self.label_end_ix.shape:
            raise ValueError('labels must be [n, L] and the pointer arrays of equal length')

    @classmethod
    def load(cls, path):
        if path.endswith('.npz'):
            z = np.load(path, allow_pickle=False)
            return cls(z['labels'], z['label_start_ix'], z['label_end_ix'])
        try:
            import h5py
        except ImportError:
            raise NotSupported('%s: reading HDF5 labels needs h5py, which is not installed; export the '
                               'labels / label_start_ix / label_end_ix arrays to an .npz' % path)
        with h5py.File(path, 'r') as f:
            return cls(f['labels'][:], f['label_start_ix'][:], f['label_end_ix'][:])

    def save_npz(self, path):
        np.savez_compressed(path, labels=self.labels, label_start_ix=self.label_start_ix,
                            label_end_ix=self.label_end_ix)


# ---------------------------------------------------------------- loader --------------------------
class CocoFcDataLoader:
    """DataLoader for the fc_caption path: `get_batch(split)` returns the reference's batch dict
    (fc_feats [B * seq_per_img, F] float32, labels [B * seq_per_img, L + 2], gts, bounds, infos),
    which `nicnes.nes.unique_batch` and the engine consume."""

    def __init__(self, input_json, input_fc_dir, labels, batch_size, seq_per_img=5, train_only=0, seed=0):
        with open(input_json) as f:
            self.info = json.load(f)
        self.ix_to_word = self.info['ix_to_word']
        self.vocab_size = len(self.ix_to_word)
        self.input_fc_dir = input_fc_dir
        self.labels = labels if isinstance(labels, LabelStore) else LabelStore.load(labels)
        self.seq_length = self.labels.labels.shape[1]
        self.batch_size = int(batch_size)
        self.seq_per_img = int(seq_per_img or 5)
        self.num_images = self.labels.label_start_ix.shape[0]
        self.rng = random.Random(seed)
        self.split_ix = {'train': [], 'val': [], 'test': []}
        for ix, img in enumerate(self.info['images']):
            sp = img.get('split')
            if sp in self.split_ix:
                self.split_ix[sp].append(ix)
            elif train_only == 0:                                   # restval
                self.split_ix['train'].append(ix)
        self.iterators = {'train': 0, 'val': 0, 'test': 0}
        self.rng.shuffle(self.split_ix['train'])                 # BlobFetcher(if_shuffle=True)

    def get_vocab(self):
        return self.ix_to_word

    def get_seq_length(self):
        return self.seq_length

    def length_of_split(self, split):
        assert split in ('train', 'val', 'test'), 'now: {}'.format(split)
        return len(self.split_ix[split])

    def fc_feature(self, ix):
        path = os.path.join(self.input_fc_dir, str(self.info['images'][ix]['id']) + '.npy')
        return np.load(path, allow_pickle=False)

    def get_captions(self, ix, seq_per_img):
        ix1 = int(self.labels.label_start_ix[ix]) - 1               # 1-based pointers
        ix2 = int(self.labels.label_end_ix[ix]) - 1
        ncap = ix2 - ix1 + 1
        assert ncap > 0, 'an image does not have any label. this can be handled but right now isn\'t'
        lab = self.labels.labels
        if ncap < seq_per_img:
            seq = np.zeros([seq_per_img, self.seq_length], dtype='int')
            for q in range(seq_per_img):
                seq[q, :] = lab[self.rng.randint(ix1, ix2), :self.seq_length]
        else:
            ixl = self.rng.randint(ix1, ix2 - seq_per_img + 1)
            seq = lab[ixl: ixl + seq_per_img, :self.seq_length]
        return seq

    def _next_ix(self, split):
        order = self.split_ix[split]
        if not order:
            raise ValueError('split %r has no images' % split)
        ri = self.iterators[split]
        ix = order[ri]
        ri_next = ri + 1
        wrapped = False
        if ri_next >= len(order):
            ri_next = 0
            if split == 'train':
                self.rng.shuffle(order)
            wrapped = True
        self.iterators[split] = ri_next
        return ix, wrapped

    def get_batch(self, split, batch_size=None, seq_per_img=None):
        batch_size = batch_size or self.batch_size
        seq_per_img = seq_per_img or self.seq_per_img
        fc_batch, gts, infos = [], [], []
        label_batch = np.zeros([batch_size * seq_per_img, self.seq_length + 2], dtype='int')
        wrapped = False
        for i in range(batch_size):
            ix, w = self._next_ix(split)
            wrapped = wrapped or w
            fc_batch.append(self.fc_feature(ix))
            label_batch[i * seq_per_img: (i + 1) * seq_per_img, 1: self.seq_length + 1] = \
                self.get_captions(ix, seq_per_img)
            gts.append(self.labels.labels[self.labels.label_start_ix[ix] - 1: self.labels.label_end_ix[ix]])
            img = self.info['images'][ix]
            infos.append({'ix': ix, 'id': img['id'], 'file_path': img.get('file_path')})
        return {'fc_feats': np.stack(sum([[f] * seq_per_img for f in fc_batch], [])).astype(np.float32),
                'labels': label_batch, 'gts': gts,
                'bounds': {'it_pos_now': self.iterators[split], 'it_max': len(self.split_ix[split]),
                           'wrapped': wrapped},
                'infos': infos}


# ---------------------------------------------------------------- df table ------------------------
class _DfUnpickler(pickle.Unpickler):
    """Builds only plain containers: the df pickle is data, never code."""
    _ALLOWED = {('collections', 'defaultdict'), ('builtins', 'float'), ('builtins', 'int'),
                ('builtins', 'dict'), ('builtins', 'tuple'), ('builtins', 'list'), ('builtins', 'str'),
                ('__builtin__', 'float'), ('__builtin__', 'int'), ('numpy', 'float64'), ('numpy.core.multiarray', 'scalar'), ('numpy', 'dtype')}

    def find_class(self, module, name):
        if (module, name) not in self._ALLOWED:
            raise pickle.UnpicklingError('df table: %s.%s is not allowed' % (module, name))
        if (module, name) == ('collections', 'defaultdict'):
            return collections.defaultdict
        if module in ('builtins', '__builtin__'):
            return {'float': float, 'int': int, 'dict': dict, 'tuple': tuple, 'list': list, 'str': str}[name]
        if (module, name) == ('numpy', 'float64'):
            return np.float64
        if (module, name) == ('numpy', 'dtype'):
            return np.dtype
        if name == 'scalar':
            from numpy.core.multiarray import scalar
            return scalar
        raise pickle.UnpicklingError('df table: %s.%s' % (module, name))


def _df_from_obj(obj):
    df = obj['document_frequency']
    return {tuple(str(w) for w in g): float(v) for g, v in dict(df).items()}, float(obj['ref_len'])


def load_df_table(path):
    """-> (document_frequency {n-gram tuple of word strings: df}, ref_len_raw). Reads the upstream
    CiderD pickle (restricted unpickler, latin1 strings as upstream opens it under Python 3), or the
    .json / .npz forms written by `save_df_table`. The scorer uses log(ref_len_raw)."""
    if path.endswith('.json'):
        with open(path) as f:
            obj = json.load(f)
        return {tuple(k.split(' ')): float(v) for k, v in obj['document_frequency'].items()}, float(obj['ref_len'])
    if path.endswith('.npz'):
        z = np.load(path, allow_pickle=False)
        keys, vals = z['keys'].astype(np.uint64), z['df']
        df = {}
        for k, v in zip(keys.tolist(), vals.tolist()):
            n = k >> 56
            df[tuple(str((k >> (42 - 14 * i)) & 0x3fff) for i in range(n))] = float(v)
        return df, float(z['ref_len'])
    with open(path, 'rb') as f:
        obj = _DfUnpickler(io.BytesIO(f.read()), encoding='latin1').load()
    return _df_from_obj(obj)


def save_df_table(path, document_frequency, ref_len_raw):
    """Portable df table: .json ({'document_frequency': {'w1 w2': df}, 'ref_len'}) or .npz (the
    packed keys of `nicnes.df_table_arrays`, df, ref_len)."""
    if path.endswith('.npz'):
        from .engine import df_table_arrays
        keys, vals = df_table_arrays(document_frequency)
        np.savez_compressed(path, keys=keys, df=vals, ref_len=np.float64(ref_len_raw))
        return
    with open(path, 'w') as f:
        json.dump({'document_frequency': {' '.join(str(w) for w in g): float(v)
                                          for g, v in document_frequency.items()},
                   'ref_len': float(ref_len_raw)}, f)


def loader_from_caption_options(exp, batch_size, seed=0, root='.'):
    """The training loader an experiment's caption_options name (input_json, input_fc_dir, input_label_h5,
    seq_per_img, train_only: captioning/experiment.py:9-44), at `batch_size`. Relative paths are taken from
    `root` (the reference runs from its src/ directory). Without h5py, an .npz export next to the .h5 (same
    stem) is read instead. Raises FileNotFoundError when the data is not there."""
    opt = dict(exp.get('caption_options') or {})
    for k in ('input_json', 'input_fc_dir', 'input_label_h5'):
        if not opt.get(k):
            raise FileNotFoundError('caption_options.%s is not set' % k)

    def path(p):
        return p if os.path.isabs(p) else os.path.join(root, p)
    labels = path(opt['input_label_h5'])
    npz = os.path.splitext(labels)[0] + '.npz'
    if not labels.endswith('.npz') and os.path.exists(npz):
        try:
            import h5py  # noqa: F401
        except ImportError:
            labels = npz
    for p in (path(opt['input_json']), path(opt['input_fc_dir']), labels):
        if not os.path.exists(p):
            raise FileNotFoundError(p)
    return CocoFcDataLoader(path(opt['input_json']), path(opt['input_fc_dir']), labels, batch_size,
                            seq_per_img=opt.get('seq_per_img') or 5, train_only=opt.get('train_only') or 0,
                            seed=seed)


def batches(loader, split='train', batch_size=None):
    """Endless batch stream for EngineMaster.run / run_dispatched, as the reference master draws one
    batch per iteration (nic_nes_master.py:80-96 via tools/iteration.py:150-192)."""
    while True:
        yield loader.get_batch(split, batch_size=batch_size)
