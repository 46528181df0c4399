"""Statistics shared by the CPU (oracle) and GPU (HIP) pins to reference-held images (test
infrastructure).  See tests/golden/make_recon_fixture.py and make_manifold_fixture.py."""
import numpy as np


def lv_head_beta(pairs):
    """Pin of the posterior spread exp(lv / 2) (VAEB.py:41-47, 271-291) against the reference's
    num_samples = 20 reconstructions.  For each model: y0 = decoder mean at z = mu,
    yE = the mean decoder output over many posterior draws (its expectation), yr0 / yr20 =
    the reference's saved num_samples = 0 / 20 outputs of the same inputs.  The sampled
    reconstruction differs from y0 by the decoder's curvature over the posterior spread,
    s = yE - y0 (a few 1e-4 per pixel); the reference's own difference r = yr20 - yr0 carries
    that shift plus noise (its 20-draw average, its two closing N(y, exp(y_log_sigma)^2)
    draws, JPEG), and the JPEG's own bias cancels in the difference.  Least squares
    r = beta s over all pixels of all models: beta ~ 1 when s has the reference's spread;
    a spread too wide (e.g. b5 + 2: s ~ e^2 larger) gives beta << 1.  Returns (beta, se)."""
    s = np.concatenate([(yE - y0).ravel() for y0, yE, _, _ in pairs]).astype(np.float64)
    r = np.concatenate([(yr20 - yr0).ravel() for _, _, yr0, yr20 in pairs]).astype(np.float64)
    ss = s @ s
    beta = (s @ r) / ss
    se = np.std(r - beta * s) / np.sqrt(ss)
    return float(beta), float(se)


def manifold_match(mu, faces):
    """(mean |mu - face|, fraction of faces nearest to their own grid point's decode)."""
    d = np.abs(mu - faces).mean()
    M = np.abs(mu[None, :, :] - faces[:, None, :]).mean(-1)
    return float(d), float((M.argmin(1) == np.arange(len(faces))).mean())
