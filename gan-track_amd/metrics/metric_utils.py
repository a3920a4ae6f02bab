"""Feature statistics for FID, per modality (SG3/metrics/metric_utils.py:23-306, restated).

Differences by design (same numbers up to float64 summation order):
  * feature moments accumulate ON THE DEVICE in float64 (sum x and x^T x as GEMMs), and ranks combine
    them with ONE all_reduce at the end; the reference broadcasts every batch's features from every rank
    to every rank and accumulates in numpy on the host (:116-126);
  * the Inception detector is not fetched from NGC (no network, and unpickling a downloaded file runs
    code): it is SUPPLIED -- `register_detector(url_or_name, module)` with any callable
    images uint8 [N, 3, H, W] -> features [N, F], or a TorchScript file path.

Kept as in the reference, because they change the numbers:
  * the real-image quirk (:240-246): a batch whose max() is not exactly 255 is multiplied by 255,
    clamped to [0, 255] and cast to uint8 -- otherwise the float [0, 255] data pass unchanged;
  * generated images: uint8(clamp(img * 127.5 + 128, 0, 255)) (:292);
  * per modality: channel `mode_idx` of the multi-channel image, repeated to 3 channels (:250-255);
  * rank r evaluates items (i * num_gpus + r) % num_items (:237); labels for G from the dataset (:62-72).
"""
import copy
import hashlib
import os
import time
import uuid

import numpy as np
import torch

import dnnlib

_detectors = {}


def register_detector(url, module):
    """Make `module` (callable: uint8 images [N,3,H,W] -> float features [N,F]) the detector for `url`."""
    _detectors[url] = module


def get_feature_detector_name(url):
    return os.path.splitext(url.split('/')[-1])[0]


def get_feature_detector(url, device=torch.device('cpu'), num_gpus=1, rank=0, verbose=False):
    det = _detectors.get(url)
    if det is None:
        path = url if os.path.isfile(url) else os.environ.get('SG2_FID_DETECTOR')
        if path is None or not os.path.isfile(path):
            raise RuntimeError(f'feature detector {url!r} is not available offline: register one with '
                               'metrics.metric_utils.register_detector() or point SG2_FID_DETECTOR at a '
                               'TorchScript file')
        det = _detectors[url] = torch.jit.load(path, map_location='cpu').eval()
    if isinstance(det, torch.nn.Module):
        det = det.to(device)
    return det


class MetricOptions:
    def __init__(self, G=None, G_kwargs={}, dataset_kwargs={}, num_gpus=1, rank=0, device=None, progress=None,
                 cache=True, mode_dict=None):
        assert 0 <= rank < num_gpus
        self.G = G
        self.G_kwargs = dnnlib.EasyDict(G_kwargs)
        self.dataset_kwargs = dnnlib.EasyDict(dataset_kwargs)
        self.num_gpus, self.rank = num_gpus, rank
        self.device = device if device is not None else torch.device('cuda', rank)
        self.progress = progress.sub() if progress is not None and rank == 0 else ProgressMonitor()
        self.cache = cache
        self.mode_dict = mode_dict


def iterate_random_labels(opts, batch_size):
    if opts.G.c_dim == 0:
        c = torch.zeros([batch_size, opts.G.c_dim], device=opts.device)
        while True:
            yield c
    dataset = dnnlib.util.construct_class_by_name(**opts.dataset_kwargs)
    while True:
        c = np.stack([dataset.get_label(np.random.randint(len(dataset))) for _ in range(batch_size)])
        yield torch.from_numpy(c).to(opts.device)


class FeatureStats:
    """Running feature moments (float64) -- mean / covariance for FID; optionally all features."""

    def __init__(self, capture_all=False, capture_mean_cov=False, max_items=None):
        self.capture_all, self.capture_mean_cov, self.max_items = capture_all, capture_mean_cov, max_items
        self.num_items = 0
        self.num_features = None
        self.all_features = None
        self.raw_mean = None      # float64 sum of x      (torch, on the features' device)
        self.raw_cov = None       # float64 sum of x x^T

    def set_num_features(self, num_features, device=None):
        if self.num_features is not None:
            assert num_features == self.num_features
            return
        self.num_features = num_features
        self.all_features = []
        self.raw_mean = torch.zeros([num_features], dtype=torch.float64, device=device)
        self.raw_cov = torch.zeros([num_features, num_features], dtype=torch.float64, device=device)

    def is_full(self):
        return self.max_items is not None and self.num_items >= self.max_items

    def append_torch(self, x, num_gpus=1, rank=0):
        """This rank's features of one batch (every rank passes the same batch size; rank r's k-th row is
        item k * num_gpus + r of the global, interleaved stream, as the reference's broadcast builds it).
        Call reduce() once after the last batch."""
        assert isinstance(x, torch.Tensor) and x.ndim == 2
        x = x.float()
        total = x.shape[0] * num_gpus                    # items this batch adds to the global stream
        if self.max_items is not None and self.num_items + total > self.max_items:
            room = max(self.max_items - self.num_items, 0)
            x = x[:max(0, (room - rank + num_gpus - 1) // num_gpus)]
            total = room
        self.set_num_features(x.shape[1], x.device)
        self.num_items += total
        if self.capture_all:
            self.all_features.append(x.cpu().numpy())
        if self.capture_mean_cov and x.shape[0]:
            x64 = x.double()
            self.raw_mean += x64.sum(0)
            self.raw_cov += x64.T @ x64

    def append(self, x):
        self.append_torch(torch.as_tensor(np.asarray(x, dtype=np.float32)))

    def reduce(self, num_gpus):
        if num_gpus > 1 and self.capture_mean_cov:
            torch.distributed.all_reduce(self.raw_mean)
            torch.distributed.all_reduce(self.raw_cov)

    def get_all(self):
        assert self.capture_all
        return np.concatenate(self.all_features, axis=0)

    def get_mean_cov(self):
        assert self.capture_mean_cov
        mean = (self.raw_mean / self.num_items).cpu().numpy()
        cov = (self.raw_cov / self.num_items).cpu().numpy()
        return mean, cov - np.outer(mean, mean)

    def save(self, path):
        np.savez(path, num_items=self.num_items, num_features=self.num_features, max_items=-1 if self.max_items is None
                 else self.max_items, raw_mean=self.raw_mean.cpu().numpy(), raw_cov=self.raw_cov.cpu().numpy())

    @staticmethod
    def load(path):
        z = np.load(path, allow_pickle=False)
        s = FeatureStats(capture_mean_cov=True, max_items=None if int(z['max_items']) < 0 else int(z['max_items']))
        s.num_items, s.num_features = int(z['num_items']), int(z['num_features'])
        s.raw_mean, s.raw_cov = torch.from_numpy(z['raw_mean']), torch.from_numpy(z['raw_cov'])
        return s


class ProgressMonitor:
    def __init__(self, tag=None, num_items=None, flush_interval=1000, verbose=False, progress_fn=None, pfn_lo=0,
                 pfn_hi=1000, pfn_total=1000):
        self.tag, self.num_items, self.verbose, self.flush_interval = tag, num_items, verbose, flush_interval
        self.progress_fn, self.pfn_lo, self.pfn_hi, self.pfn_total = progress_fn, pfn_lo, pfn_hi, pfn_total
        self.start_time = self.batch_time = time.time()
        self.batch_items = 0
        if progress_fn is not None:
            progress_fn(pfn_lo, pfn_total)

    def update(self, cur_items):
        if cur_items < self.batch_items + self.flush_interval and (self.num_items is None or cur_items < self.num_items):
            return
        now = time.time()
        if self.verbose and self.tag is not None:
            print(f'{self.tag:<19s} items {cur_items:<7d} time {dnnlib.util.format_time(now - self.start_time):<12s}')
        self.batch_time, self.batch_items = now, cur_items
        if self.progress_fn is not None and self.num_items is not None:
            self.progress_fn(self.pfn_lo + (self.pfn_hi - self.pfn_lo) * (cur_items / self.num_items), self.pfn_total)

    def sub(self, tag=None, num_items=None, flush_interval=1000, rel_lo=0, rel_hi=1):
        return ProgressMonitor(tag, num_items, flush_interval, self.verbose, self.progress_fn,
                               self.pfn_lo + (self.pfn_hi - self.pfn_lo) * rel_lo,
                               self.pfn_lo + (self.pfn_hi - self.pfn_lo) * rel_hi, self.pfn_total)


def _select_mode(images, mode_dict):
    x = images[:, mode_dict['mode_idx']].unsqueeze(1) if mode_dict is not None else images
    return x.repeat([1, 3, 1, 1]) if x.shape[1] == 1 else x


def real_images_to_uint8_quirk(images):
    """The reference's real-side conversion (metric_utils.py:240-246), per batch."""
    if images.max() != 255:
        return (images * 255).clamp(0, 255).to(torch.uint8)
    return images


def compute_feature_stats_for_dataset(opts, detector_url, detector_kwargs, mode_dict, rel_lo=0, rel_hi=1, batch_size=64,
                                      data_loader_kwargs=None, max_items=None, **stats_kwargs):
    dataset = dnnlib.util.construct_class_by_name(**opts.dataset_kwargs)
    cache_file = None
    if opts.cache:
        args = dict(dataset_kwargs=opts.dataset_kwargs, detector_url=detector_url, detector_kwargs=detector_kwargs,
                    stats_kwargs=stats_kwargs)
        md5 = hashlib.md5(repr(sorted(args.items())).encode('utf-8'))
        tag = f"{dataset.name}-{mode_dict['mode_name'] if mode_dict else 'all'}-{get_feature_detector_name(detector_url)}-{md5.hexdigest()}"
        cache_file = dnnlib.make_cache_dir_path('gan-metrics', tag + '.npz')
        flag = os.path.isfile(cache_file) if opts.rank == 0 else False
        if opts.num_gpus > 1:
            f = torch.as_tensor(float(flag), dtype=torch.float32, device=opts.device)
            torch.distributed.broadcast(f, src=0)
            flag = float(f.cpu()) != 0
        if flag:
            return FeatureStats.load(cache_file)
    num_items = len(dataset) if max_items is None else min(len(dataset), max_items)
    stats = FeatureStats(max_items=num_items, **stats_kwargs)
    progress = opts.progress.sub(tag='dataset features', num_items=num_items, rel_lo=rel_lo, rel_hi=rel_hi)
    detector = get_feature_detector(detector_url, device=opts.device, num_gpus=opts.num_gpus, rank=opts.rank)
    subset = [(i * opts.num_gpus + opts.rank) % num_items for i in range((num_items - 1) // opts.num_gpus + 1)]
    # a DataLoader as in the reference (:248): besides batching, creating its iterator draws one value from
    # torch's global generator, so the generator pass that follows sees the reference's latents
    if data_loader_kwargs is None:
        data_loader_kwargs = dict(pin_memory=True, num_workers=3, prefetch_factor=2)
    for imgs, _labels, _names in torch.utils.data.DataLoader(dataset=dataset, sampler=subset, batch_size=batch_size,
                                                             **data_loader_kwargs):
        imgs = real_images_to_uint8_quirk(imgs)
        feats = detector(_select_mode(imgs, mode_dict).to(opts.device), **detector_kwargs)
        stats.append_torch(feats, num_gpus=opts.num_gpus, rank=opts.rank)
        progress.update(stats.num_items)
    stats.reduce(opts.num_gpus)
    if cache_file is not None and opts.rank == 0:
        os.makedirs(os.path.dirname(cache_file), exist_ok=True)
        tmp = cache_file + '.' + uuid.uuid4().hex + '.npz'
        stats.save(tmp)
        os.replace(tmp, cache_file)
    return stats


def compute_feature_stats_for_generator(opts, detector_url, detector_kwargs, mode_dict, rel_lo=0, rel_hi=1, batch_size=64,
                                        batch_gen=None, **stats_kwargs):
    batch_gen = min(batch_size, 4) if batch_gen is None else batch_gen
    assert batch_size % batch_gen == 0
    G = copy.deepcopy(opts.G).eval().requires_grad_(False).to(opts.device)
    c_iter = iterate_random_labels(opts, batch_gen)
    stats = FeatureStats(**stats_kwargs)
    assert stats.max_items is not None
    progress = opts.progress.sub(tag='generator features', num_items=stats.max_items, rel_lo=rel_lo, rel_hi=rel_hi)
    detector = get_feature_detector(detector_url, device=opts.device, num_gpus=opts.num_gpus, rank=opts.rank)
    while not stats.is_full():
        imgs = []
        for _ in range(batch_size // batch_gen):
            z = torch.randn([batch_gen, G.z_dim], device=opts.device)
            img = G(z=z, c=next(c_iter), **opts.G_kwargs)
            imgs.append((img.float() * 127.5 + 128).clamp(0, 255).to(torch.uint8))
        feats = detector(_select_mode(torch.cat(imgs), mode_dict), **detector_kwargs)
        stats.append_torch(feats, num_gpus=opts.num_gpus, rank=opts.rank)
        progress.update(stats.num_items)
    stats.reduce(opts.num_gpus)
    return stats
