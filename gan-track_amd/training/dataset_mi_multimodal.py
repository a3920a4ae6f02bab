"""Claro / Pelvis training data: a zip of per-slice pickles, served from HBM.

Drop-in for SG3/training/dataset_mi_multimodal.py:30-285 (`Dataset`, `CustomImageFolderDataset`; the
class-name string `training.dataset_mi_multimodal.CustomImageFolderDataset` of the reference's
training_options resolves here).  On-disk format (written by src/data/dataset_tool_mi.py:625-714,839-860):

    <zip>/<split>/<patient>/<patient>_<slice:05d>.pickle   dict {modality: HxW array in [0, 255]}
    <zip>/<split>/dataset.json                              {"labels": [[relpath, label], ...]} or null

An item is the CHW float32 stack of the requested modalities (channel = modality, in the given order),
its label (int -> one-hot float32), and its file name -- the reference's `__getitem__` (:106-116),
including max_size (:61-64) and the x-flip doubling (:67-70, mirrored left-right).

Two things differ by design:
  * the pickles are read with `SafeUnpickler`, which reconstructs plain containers and numpy arrays and
    refuses everything else (a pickle is code; a training set should not be able to run any);
  * `DeviceImageCache` decodes the whole split ONCE into one float32 tensor resident in HBM (a Claro
    split is a few GB; an MI355X has 288 GB), after which a training batch is an index gather on the
    device plus the reference's `/127.5 - 1` (training_loop_mi_multimodal.py:317) -- no per-step
    unpickling, no host->device image copies.  At MI355X step rates the reference's 3-worker
    pickle-per-slice DataLoader would be the bottleneck.  Batches follow the reference sampler's order
    (torch_utils/misc.py InfiniteSampler, rank-strided), so the data stream is the reference's.
"""
import io
import json
import os
import pickle
import zipfile

import numpy as np
import torch

import dnnlib
from torch_utils import misc


class SafeUnpickler(pickle.Unpickler):
    """Unpickles only builtin containers / scalars and numpy arrays, dtypes and scalars."""

    _ALLOWED = {
        ('builtins', 'dict'), ('builtins', 'list'), ('builtins', 'tuple'), ('builtins', 'set'),
        ('builtins', 'frozenset'), ('builtins', 'int'), ('builtins', 'float'), ('builtins', 'complex'),
        ('builtins', 'bool'), ('builtins', 'str'), ('builtins', 'bytes'), ('builtins', 'bytearray'),
        ('collections', 'OrderedDict'), ('numpy', 'ndarray'), ('numpy', 'dtype'),
        ('numpy.core.multiarray', '_reconstruct'), ('numpy.core.multiarray', 'scalar'),
        ('numpy._core.multiarray', '_reconstruct'), ('numpy._core.multiarray', 'scalar'),
        ('numpy.core.numeric', '_frombuffer'), ('numpy._core.numeric', '_frombuffer'),
    }

    def find_class(self, module, name):
        if (module, name) in self._ALLOWED:
            return super().find_class(module, name)
        if module == 'numpy' and name in ('float16', 'float32', 'float64', 'uint8', 'int16', 'int32', 'int64',
                                          'uint16', 'bool_'):
            return getattr(np, name)
        raise pickle.UnpicklingError(f'dataset pickle refers to {module}.{name}: not a plain array / dict; refused')


def safe_load_pickle(f):
    return SafeUnpickler(f).load()


class Dataset(torch.utils.data.Dataset):
    """Reference base class semantics (SG3/training/dataset_mi_multimodal.py:30-188)."""

    def __init__(self, name, raw_shape, dtype, max_size=None, use_labels=False, xflip=False, split='train',
                 modalities=None, random_seed=0):
        self._name = name
        self._dtype = dtype
        self._split = split
        self._modalities = list(modalities) if modalities is not None else ['MR_nonrigid_CT', 'MR_MR_T2']
        self._raw_shape = list(raw_shape)
        self._use_labels = use_labels
        self._raw_labels = None
        self._label_shape = None
        self._raw_idx = np.arange(self._raw_shape[0], dtype=np.int64)
        if max_size is not None and self._raw_idx.size > max_size:
            np.random.RandomState(random_seed).shuffle(self._raw_idx)
            self._raw_idx = np.sort(self._raw_idx[:max_size])
        self._xflip = np.zeros(self._raw_idx.size, dtype=np.uint8)
        if xflip:
            self._raw_idx = np.tile(self._raw_idx, 2)
            self._xflip = np.concatenate([self._xflip, np.ones_like(self._xflip)])

    def _get_raw_labels(self):
        if self._raw_labels is None:
            self._raw_labels = self._load_raw_labels() if self._use_labels else None
            if self._raw_labels is None:
                self._raw_labels = np.zeros([self._raw_shape[0], 0], dtype=np.float32)
            assert isinstance(self._raw_labels, np.ndarray) and self._raw_labels.shape[0] == self._raw_shape[0]
            assert self._raw_labels.dtype in (np.float32, np.int64)
            if self._raw_labels.dtype == np.int64:
                assert self._raw_labels.ndim == 1 and np.all(self._raw_labels >= 0)
        return self._raw_labels

    def close(self):
        pass

    def _load_raw_image(self, raw_idx):
        raise NotImplementedError

    def _load_raw_labels(self):
        raise NotImplementedError

    def __getstate__(self):
        return dict(self.__dict__, _raw_labels=None)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __len__(self):
        return self._raw_idx.size

    def __getitem__(self, idx):
        image, fname = self._load_raw_image(self._raw_idx[idx])
        assert isinstance(image, np.ndarray) and list(image.shape) == self.image_shape
        assert image.dtype == self._dtype
        if self._xflip[idx]:
            image = image[:, :, ::-1]
        return image.copy(), self.get_label(idx), fname

    def get_label(self, idx):
        label = self._get_raw_labels()[self._raw_idx[idx]]
        if label.dtype == np.int64:
            onehot = np.zeros(self.label_shape, dtype=np.float32)
            onehot[label] = 1
            label = onehot
        return label.copy()

    def get_details(self, idx):
        d = dnnlib.EasyDict()
        d.raw_idx = int(self._raw_idx[idx])
        d.xflip = int(self._xflip[idx]) != 0
        d.raw_label = self._get_raw_labels()[d.raw_idx].copy()
        return d

    name = property(lambda self: self._name)
    dtype = property(lambda self: self._dtype)
    modatilies = property(lambda self: self._modalities)     # (sic) the reference's property name
    modalities = property(lambda self: self._modalities)
    split = property(lambda self: self._split)
    image_shape = property(lambda self: list(self._raw_shape[1:]))

    @property
    def num_channels(self):
        assert len(self.image_shape) == 3
        return self.image_shape[0]

    @property
    def resolution(self):
        assert len(self.image_shape) == 3 and self.image_shape[1] == self.image_shape[2]
        return self.image_shape[1]

    @property
    def label_shape(self):
        if self._label_shape is None:
            raw = self._get_raw_labels()
            self._label_shape = [int(np.max(raw)) + 1] if raw.dtype == np.int64 else raw.shape[1:]
        return list(self._label_shape)

    @property
    def label_dim(self):
        assert len(self.label_shape) == 1
        return self.label_shape[0]

    @property
    def has_labels(self):
        return any(x != 0 for x in self.label_shape)

    @property
    def has_onehot_labels(self):
        return self._get_raw_labels().dtype == np.int64


class CustomImageFolderDataset(Dataset):
    """Zip of per-slice pickles (SG3/training/dataset_mi_multimodal.py:193-285)."""

    def __init__(self, path, resolution=None, **super_kwargs):
        self._path = path
        self._zipfile = None
        self._split = super_kwargs['split']
        self._modalities = list(super_kwargs['modalities'])
        if os.path.splitext(path)[1].lower() != '.zip':
            raise IOError('Path must point to a directory or zip')
        self._type = 'zip'
        self._all_fnames = set(self._get_zipfile().namelist())
        self._image_fnames = sorted(f for f in self._all_fnames
                                    if os.path.splitext(f)[1].lower() == '.pickle' and self._split in f)
        if not self._image_fnames:
            raise IOError('No image files found in the specified path')
        name = os.path.splitext(os.path.basename(path))[0]
        raw_shape = [len(self._image_fnames)] + list(self._load_raw_image(0)[0].shape)
        if resolution is not None and (raw_shape[2] != resolution or raw_shape[3] != resolution):
            raise IOError('Image files do not match the specified resolution')
        super().__init__(name=name, raw_shape=raw_shape, **super_kwargs)

    def _get_zipfile(self):
        if self._zipfile is None:
            self._zipfile = zipfile.ZipFile(self._path)
        return self._zipfile

    def close(self):
        try:
            if self._zipfile is not None:
                self._zipfile.close()
        finally:
            self._zipfile = None

    def __getstate__(self):
        return dict(super().__getstate__(), _zipfile=None)

    def _load_raw_image(self, raw_idx):
        fname = self._image_fnames[raw_idx]
        with self._get_zipfile().open(fname, 'r') as f:
            slices = safe_load_pickle(io.BytesIO(f.read()))
        first = np.asarray(slices[self._modalities[0]])
        out = np.zeros((len(self._modalities), first.shape[0], first.shape[1]), dtype=np.float32)
        for i, m in enumerate(self._modalities):
            out[i] = np.asarray(slices[m]).astype(np.float32)
        return out, fname

    def _load_raw_labels(self):
        fname = f'{self._split}/dataset.json'
        if fname not in self._all_fnames:
            return None
        with self._get_zipfile().open(fname, 'r') as f:
            labels = json.load(f)['labels']
        if labels is None:
            return None
        labels = dict(labels)
        labels = [labels[os.path.relpath(fn.replace('\\', '/'), f'{self._split}/')] for fn in self._image_fnames]
        labels = np.array(labels)
        return labels.astype({1: np.int64, 2: np.float32}[labels.ndim])


class DeviceImageCache:
    """The whole (max_size-limited) split decoded once into HBM; yields the training loop's batches.

    next(cache) -> (images [B, C, H, W] float32 in [-1, 1] on `device`, labels [B, c_dim] float32), the
    samples drawn in the order of InfiniteSampler(dataset, rank, num_replicas, seed) exactly as the
    reference's DataLoader would batch them (training_loop_mi_multimodal.py:178-179, 313-318).  The
    x-flipped half of an xflip dataset is a flip on the device, not a second copy."""

    def __init__(self, dataset, device, batch_size, rank=0, num_replicas=1, seed=0):
        self.dataset = dataset
        self.device = torch.device(device)
        self.batch_size = batch_size
        raw_ids = np.unique(dataset._raw_idx)
        slot = {int(r): i for i, r in enumerate(raw_ids)}
        imgs = torch.empty([len(raw_ids)] + dataset.image_shape, dtype=torch.float32)
        for i, r in enumerate(raw_ids):
            imgs[i] = torch.from_numpy(dataset._load_raw_image(int(r))[0])
        self.images = imgs.to(self.device)
        self.slots = torch.tensor([slot[int(r)] for r in dataset._raw_idx], dtype=torch.int64, device=self.device)
        self.flip = torch.from_numpy(dataset._xflip.astype(np.bool_)).to(self.device)
        self.labels = torch.from_numpy(np.stack([dataset.get_label(i) for i in range(len(dataset))])
                                       if len(dataset) else np.zeros([0, 0], np.float32)).to(self.device)
        self._order = iter(misc.InfiniteSampler(dataset, rank=rank, num_replicas=num_replicas, seed=seed))

    def __iter__(self):
        return self

    def next_indices(self):
        return [next(self._order) for _ in range(self.batch_size)]

    def __next__(self):
        idx = torch.tensor(self.next_indices(), dtype=torch.int64).to(self.device, non_blocking=True)
        img = self.images.index_select(0, self.slots.index_select(0, idx))
        img = torch.where(self.flip.index_select(0, idx)[:, None, None, None], img.flip(3), img)
        return img / 127.5 - 1, self.labels.index_select(0, idx)
