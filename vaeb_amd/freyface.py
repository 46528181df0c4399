"""Drop-in for the reference's freyFace.py (/root/reference/freyFace.py): its `VAE` class
(:32-267) and the 10 x 10 latent-manifold driver (:311-369).

freyFace.VAE trains exactly as VAEBfullbayes.VAE (same single-draw initialisation :42-124,
one eps per step :199-203, mean objective :212, Adagrad + -lr*1e-6*theta^2 :257-263) and adds
(i) the trained model: when `modelFrey.pkl` (continuous) / `modelMNIST.pkl` (Bernoulli) is in
the working directory its parameter list replaces the initialisation (:50-80), and (ii) the
compiled decoder `freyFace(z)` (:173-187, 237-245) that the driver evaluates on the grid
z = [Phi^-1((ii + 0.9) / 10), Phi^-1((jj + 0.9) / 10)].  The decoder runs in libvaeb_hip.so
(vaeb_decode); there is no CPU fallback.  Pickles are read by vaeb_amd.pickle_static, which
executes nothing from the file.
"""
from __future__ import annotations

import os

import numpy as np

from . import pickle_static
from .fullbayes import VAE as _FullBayesVAE
from .image import multiple_images, save_image

# freyFace.py:20-30
command_line_args = {"seed": (10, int), "n_latent": (2, int), "n_epochs": (2000, int), "batch_size": (100, int),
                     "L": (1, int), "hidden_unit": (-1, int), "learning_rate": (0.01, float), "trace_file": ("", str)}
command_line_flags = ["continuous"]


class VAE(_FullBayesVAE):
    """`freyFace.VAE(x_train, continuous, hidden_units, latent_size, batch_size, L,
    learning_rate)` (freyFace.py:33-34): update(index), validate(x) and freyFace(z)."""

    def __init__(self, x_train, continuous, hidden_units, latent_size, batch_size, L, learning_rate, **kw):
        name = "modelFrey.pkl" if continuous else "modelMNIST.pkl"
        params = kw.pop("params", None)
        if params is None and os.path.isfile("modelFrey.pkl"):
            # freyFace.py:50-80 tests for modelFrey.pkl, then reads the file of the decoder type
            params = pickle_static.read_array_pickle(name)
        super().__init__(x_train, continuous, hidden_units, latent_size, batch_size, L, learning_rate,
                         params=params, **kw)

    def freyFace(self, z):
        """freyFace.py:237-245: [mu, log_sigma] (continuous) or y at latents z [n x n_latent]."""
        mu, ls = self._ctx.decode(np.atleast_2d(np.asarray(z, np.float32)))
        if self.continuous:
            return [mu.astype(np.float64), ls.astype(np.float64)]
        return mu.astype(np.float64)


def manifold_grid(steps=10):
    """freyFace.py:352-354: z[ii, jj] = [Phi^-1((ii + 0.9) / 10), Phi^-1((jj + 0.9) / 10)]."""
    from scipy.stats import norm
    g = norm.ppf((np.arange(steps) + 0.9) / 10.0)
    return np.array([[g[ii], g[jj]] for ii in range(steps) for jj in range(steps)])


def draw_manifold(model, out_dir=".", rng=None):
    """freyFace.py:349-369: decode the grid, draw each continuous face from
    N(mu, exp(log_sigma)^2 I) (per pixel, same distribution as :358-361), save
    FREY{ii}{jj}.jpg (or MNIST{ii}{jj}.jpg: the Bernoulli means) and the MNIST mosaic (:369).
    All 100 grid points go through ONE vaeb_decode call.  Returns the [100 x D] images."""
    rng = np.random if rng is None else rng
    z = manifold_grid()
    out = model.freyFace(z)
    if model.continuous:
        mu, ls = out
        faces = mu + np.exp(ls) * rng.standard_normal(mu.shape)
        prefix = "FREY"
    else:
        faces = out
        prefix = "MNIST"
    for k in range(100):
        save_image(faces[k], os.path.join(out_dir, f"{prefix}{k // 10}{k % 10}.jpg"))
    if not model.continuous:
        multiple_images(os.path.join(out_dir, "MNIST"))
    return faces


def main(argv=None, data=None, out_dir="freyFaces", out=print, **kw):
    """freyFace.py's __main__ (:311-369) with the reference's parse_args / print_args.  The
    reference overrides the parsed flag with `continuous = False` (:326); here the
    -continuous flag is honoured (that override makes its own FREY*.jpg outputs, which a
    continuous run wrote, unreproducible).  `data` = (x_train, x_valid) skips the pickles."""
    from .cli import parse_args, print_args
    args = parse_args(argv, command_line_args, command_line_flags, flag_prefix='-')
    print_args(args, out)
    np.random.seed(args["seed"])
    continuous = args["continuous"]
    out("loading data")
    if data is None:
        from .cli import load_dataset
        data = load_dataset(continuous)
    x_train = data[0]
    hidden = args["hidden_unit"] if args["hidden_unit"] >= 0 else (200 if continuous else 500)
    out("creating the model")
    model = VAE(x_train, continuous, hidden, args["n_latent"], args["batch_size"], args["L"], args["learning_rate"],
                **kw)
    os.makedirs(out_dir, exist_ok=True)
    draw_manifold(model, out_dir)
    return model
