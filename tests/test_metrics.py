"""metrics.ssim_legacy: properties of SSIM (skimage absent: parity unpinned)."""
import numpy as np

from codenerf_amd.metrics import psnr, ssim_legacy


def test_ssim_identity_and_range():
    rng = np.random.default_rng(0)
    a = rng.random((32, 40, 3))
    assert abs(ssim_legacy(a, a) - 1.0) < 1e-12
    b = np.clip(a + rng.normal(0, 0.1, a.shape), 0, 1)
    s = ssim_legacy(a, b)
    assert 0.0 < s < 1.0
    # symmetric, and more noise -> lower SSIM
    assert abs(s - ssim_legacy(b, a)) < 1e-12
    c = np.clip(a + rng.normal(0, 0.3, a.shape), 0, 1)
    assert ssim_legacy(a, c) < s


def test_ssim_constant_images_closed_form():
    # constant images x = p, y = q: variances 0 -> SSIM = (2pq + C1) / (p^2 + q^2 + C1)
    C1 = (0.01 * 2.0) ** 2
    a = np.full((16, 16, 3), 0.3)
    b = np.full((16, 16, 3), 0.5)
    expect = (2 * 0.3 * 0.5 + C1) / (0.09 + 0.25 + C1)
    assert abs(ssim_legacy(a, b) - expect) < 1e-12


def test_psnr():
    assert abs(psnr(1e-2) - 20.0) < 1e-12
