"""Frechet Inception Distance (SG3/metrics/frechet_inception_distance.py:24-43): feature means and
covariances of real and generated images, FID = |mu_g - mu_r|^2 + tr(S_g + S_r - 2 sqrtm(S_g S_r))."""
import numpy as np
import scipy.linalg

from . import metric_utils

DETECTOR_URL = 'https://api.ngc.nvidia.com/v2/models/nvidia/research/stylegan3/versions/1/files/metrics/inception-2015-12-05.pkl'


def fid_from_stats(mu_gen, sigma_gen, mu_real, sigma_real):
    m = np.square(mu_gen - mu_real).sum()
    s, _ = scipy.linalg.sqrtm(np.dot(sigma_gen, sigma_real), disp=False)
    return float(np.real(m + np.trace(sigma_gen + sigma_real - s * 2)))


def compute_fid(opts, max_real, num_gen):
    detector_kwargs = dict(return_features=True)      # raw pool features, before the softmax
    mu_real, sigma_real = metric_utils.compute_feature_stats_for_dataset(
        opts=opts, detector_url=DETECTOR_URL, detector_kwargs=detector_kwargs, mode_dict=opts.mode_dict,
        rel_lo=0, rel_hi=0, capture_mean_cov=True, max_items=max_real).get_mean_cov()
    mu_gen, sigma_gen = metric_utils.compute_feature_stats_for_generator(
        opts=opts, detector_url=DETECTOR_URL, detector_kwargs=detector_kwargs, mode_dict=opts.mode_dict,
        rel_lo=0, rel_hi=1, capture_mean_cov=True, max_items=num_gen).get_mean_cov()
    if opts.rank != 0:
        return float('nan')
    return fid_from_stats(mu_gen, sigma_gen, mu_real, sigma_real)
