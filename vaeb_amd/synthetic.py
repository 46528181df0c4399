"""Synthetic stand-ins for the datasets the reference reads (mnist.pkl.gz, freyfaces.pkl
are absent from the snapshot, /root/reference/.MISSING_LARGE_BLOBS).  Shapes and value
ranges follow SURVEY 8(d)."""
import numpy as np


def mnist_like(n=60000, D=784, seed=0):
    """Binary pixels x = (U < p_d), p_d ~ Beta(0.2, 1.3) per pixel (mean ~0.13)."""
    p = np.random.default_rng(1).beta(0.2, 1.3, size=D).astype(np.float32)
    return (np.random.default_rng(seed).random((n, D), dtype=np.float32) < p).astype(np.float32)


def frey_like(n=1965, D=560, seed=2):
    """Continuous [0, 1] pixels, Beta(2, 2)."""
    return np.random.default_rng(seed).beta(2.0, 2.0, size=(n, D)).astype(np.float32)


def synth_like(n, D=4096, seed=3):
    """Config-5 roofline stress input: Bernoulli(0.5) pixels."""
    return (np.random.default_rng(seed).random((n, D), dtype=np.float32) < 0.5).astype(np.float32)
