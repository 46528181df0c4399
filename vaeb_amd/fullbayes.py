"""Drop-in for the reference's `VAEBfullbayes.VAE` (/root/reference/VAEBfullbayes.py:13-201)
and its `__main__` driver (:203-244).

Despite the file name the reference model has no weight posterior: it is the VAEB network
with (i) its own initialisation -- RandomState(10), each weight drawn ONCE in the order W3,
W4, W5, W1, W2, (W6) (:28-67), where VAEB.py draws W3 and W4 twice -- (ii) one eps draw per
step of shape mu.shape, L ignored (:129-133), (iii) the MEAN objective mean_b(KL + log p)
(:139-142) with no -1/2 sum theta^2 prior, and (iv) Adagrad with an extra -lr*1e-6*theta^2
MAP term (:178-185).  `validate(x)` returns that mean over the rows of x (:161-165).

The step runs in libvaeb_hip.so (objective VAEB_OBJ_MEAN_MAP, estimator LB, L = 1); there
is no CPU fallback.
"""
from __future__ import annotations

import time

import numpy as np

from . import _lib
from .model import SharedParam, TheanoStreamEmulation, param_shapes


def initial_params_fullbayes(D, H, Z, continuous):
    """VAEBfullbayes.py:23-73: RandomState(10), normal(0, 0.01) cast to float32, each
    weight drawn once in the order W3, W4, W5, W1, W2, (W6); zero biases; returned in the
    parameter-list order (:69-73)."""
    prng = np.random.RandomState(10)
    w = lambda a, b: prng.normal(0, 0.01, (a, b)).astype(np.float32)
    vals = {"W3": w(D, H), "W4": w(H, Z), "W5": w(H, Z), "W1": w(Z, H), "W2": w(H, D)}
    if continuous:
        vals["W6"] = w(H, D)
    return [vals[n] if n in vals else np.zeros(s, np.float32) for n, s in param_shapes(D, H, Z, continuous)]


class VAE:
    """`VAEBfullbayes.VAE(x_train, continuous=False, hidden_units=500, latent_size=10,
    batch_size=100, L=1, learning_rate=0.01)` (VAEBfullbayes.py:14-15).

    Attributes as the reference's: N, input_size, n_hidden_units, n_latent, continuous,
    learning_rate, batch_size, prng, sigmaInit, L, params (W3, W4, W5, W1, W2, [W6], b3,
    b4, b5, b1, b2, [b6]), ADA; `update(index) -> mean SGVB of batch index`,
    `validate(x) -> mean SGVB over x`.

    Keyword-only extras (not in the reference): device, rng ("philox": on-device
    counter-based normals; "theano": host emulation of the single RandomStreams op),
    seed, use_graph, max_eval_rows, params (start from given values instead of the
    reference initialisation)."""

    def __init__(self, x_train, continuous=False, hidden_units=500, latent_size=10, batch_size=100, L=1,
                 learning_rate=0.01, *, device=0, rng="philox", seed=10, use_graph=True, max_eval_rows=10000,
                 params=None):
        x_train = np.asarray(x_train, np.float32)
        self.N, self.input_size = x_train.shape
        self.n_hidden_units = hidden_units
        self.n_latent = latent_size
        self.continuous = bool(continuous)
        self.learning_rate = learning_rate
        self.batch_size = batch_size
        self.prng = np.random.RandomState(10)
        self.sigmaInit = 0.01
        self.L = L   # stored, never used by the reference's graph (one eps draw, :130)
        self._ctx = _lib.Context(self.input_size, hidden_units, latent_size, batch_size, L=1,
                                 decoder=_lib.DEC_GAUSSIAN if self.continuous else _lib.DEC_BERNOULLI,
                                 estimator=_lib.EST_LB, objective=_lib.OBJ_MEAN_MAP, lr=learning_rate,
                                 adagrad_eps=1e-6, device=device, max_eval_rows=max_eval_rows,
                                 use_graph=use_graph)
        self._shapes = param_shapes(self.input_size, hidden_units, latent_size, self.continuous)
        if params is None:
            arrs = initial_params_fullbayes(self.input_size, hidden_units, latent_size, self.continuous)
        else:
            arrs = [np.asarray(p.get_value() if hasattr(p, "get_value") else p, np.float32).reshape(s)
                    for p, (_, s) in zip(params, self._shapes)]
        self._ctx.set_params(np.concatenate([a.ravel() for a in arrs]))
        self.params = [SharedParam(self, i, n, s) for i, (n, s) in enumerate(self._shapes)]
        self._ctx.set_data(x_train)
        self.rng = rng
        if rng == "theano":
            self._stream = TheanoStreamEmulation(1, seed)   # one srng.normal op (:129-130)
            self._ctx.set_eps_mode(_lib.EPS_HOST, seed)
        else:
            self._stream = None
            self._ctx.set_eps_mode(_lib.EPS_PHILOX, seed)

    def _param_arrays(self):
        flat = self._ctx.get_params()
        out, o = [], 0
        for _, s in self._shapes:
            n = int(np.prod(s))
            out.append(flat[o:o + n].reshape(s).copy())
            o += n
        return out

    @property
    def ADA(self):
        acc = self._ctx.get_adagrad_state()
        out, o = [], 0
        for _, s in self._shapes:
            n = int(np.prod(s))
            out.append(acc[o:o + n].reshape(s))
            o += n
        return out

    def update(self, index):
        """`update(index)` (VAEBfullbayes.py:151-158): one Adagrad + MAP step on rows
        [index*B, (index+1)*B); returns mean_b(KL + log p) of that minibatch."""
        if self._stream is not None:
            self._ctx.push_eps(self._stream.draw(self.batch_size, self.n_latent))
        return self._ctx.update(int(index))

    def update_epoch(self, batch_order):
        """All steps of batch_order without a per-step host sync; returns the sum of
        their update() values (what the reference's loop accumulates, :236-238)."""
        if self._stream is not None:
            return float(sum(self.update(int(b)) for b in batch_order))
        self._ctx.epoch_elbo()   # drop anything earlier update() calls accumulated
        self._ctx.update_many(np.asarray(batch_order, np.int32))
        s, _ = self._ctx.epoch_elbo()
        return s

    def validate(self, x):
        """`validate(x)` (VAEBfullbayes.py:161-165): mean_b(KL + log p) over the rows of x."""
        x = np.asarray(x, np.float32)
        if self._stream is not None:
            self._ctx.push_eps(self._stream.draw(x.shape[0], self.n_latent))
        return self._ctx.validate(x) / x.shape[0]

    def close(self):
        self._ctx.close()


def main(n_epochs=2000, continuous=True, n_latent=10, data=None, out=print, **kw):
    """The reference's `__main__` (VAEBfullbayes.py:203-244): np.random.seed(10), Frey
    (hidden 200) or MNIST (hidden 500), per epoch a shuffled batch order, the mean of the
    batch values, then validation.  `data` = (x_train, x_valid) overrides the pickles."""
    np.random.seed(10)
    out("loading data")
    if data is None:
        from .cli import load_dataset
        data = load_dataset(continuous)
    x_train, x_valid = data
    hu_N = 200 if continuous else 500
    out("creating the model")
    model = VAE(x_train, continuous, hu_N, n_latent, **kw)
    out("learning")
    batch_order = np.arange(int(model.N / model.batch_size))
    trace = []
    epoch = 0
    while epoch < n_epochs:
        epoch += 1
        start = time.time()
        np.random.shuffle(batch_order)
        LB = model.update_epoch(batch_order) / len(batch_order)
        out("Epoch %s : [Lower bound: %s, time: %s]" % (epoch, LB, time.time() - start))
        LBvalidation = model.validate(x_valid)
        out("          [Lower bound on validation set: %s]" % LBvalidation)
        trace.append((LB, LBvalidation))
    return model, trace
