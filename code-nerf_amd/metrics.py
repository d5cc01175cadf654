"""Evaluation metrics of the reference's optimisation loop (src/optimizer.py).

``psnr(mse) = -10 log10(mse)`` (src/optimizer.py:163,169, src/trainer.py:99).

``ssim_legacy`` restates what ``skimage.metrics.structural_similarity(a, b,
multichannel=True)`` computes for the float images the reference passes
(src/optimizer.py:156; skimage is not installed here, so this is PARITY
UNPINNED -- it follows skimage's published algorithm as of the 0.18/0.19
series the reference's environment resolves to): per channel, 7x7 uniform
window (scipy.ndimage.uniform_filter, mode 'reflect'), sample covariance
(N/(N-1)), K1 = 0.01, K2 = 0.03, data_range = 2 (the float dtype range
(-1, 1) skimage infers when none is given), mean over the image cropped by
(win-1)/2 on each side, then the mean over channels; float64 throughout.
"""
import numpy as np


def psnr(mse):
    return -10.0 * np.log(mse) / np.log(10.0)


def _ssim_channel(x, y, win=7, K1=0.01, K2=0.03, data_range=2.0):
    from scipy.ndimage import uniform_filter
    npix = win * win
    cov_norm = npix / (npix - 1.0)
    ux, uy = uniform_filter(x, size=win), uniform_filter(y, size=win)
    uxx, uyy, uxy = uniform_filter(x * x, size=win), uniform_filter(y * y, size=win), uniform_filter(x * y, size=win)
    vx, vy, vxy = cov_norm * (uxx - ux * ux), cov_norm * (uyy - uy * uy), cov_norm * (uxy - ux * uy)
    C1, C2 = (K1 * data_range) ** 2, (K2 * data_range) ** 2
    S = ((2 * ux * uy + C1) * (2 * vxy + C2)) / ((ux * ux + uy * uy + C1) * (vx + vy + C2))
    pad = (win - 1) // 2
    return S[pad:-pad, pad:-pad].mean()


def ssim_legacy(img1, img2, win=7, data_range=2.0):
    """img1, img2: (H, W, C) float arrays -> mean SSIM over channels."""
    a = np.asarray(img1, dtype=np.float64)
    b = np.asarray(img2, dtype=np.float64)
    if a.shape != b.shape or a.ndim != 3:
        raise ValueError("ssim_legacy expects two (H, W, C) images of the same shape")
    return float(np.mean([_ssim_channel(a[..., c], b[..., c], win, data_range=data_range)
                          for c in range(a.shape[-1])]))
