"""Host-side mirror of the reference's `VAEB` class (/root/reference/VAEB.py:49-469).

The constructor signature, attributes and the `update(index)` / `validate(x)` contract
are the reference's; the compute runs in libvaeb_hip.so (hand-written gfx950 kernels)
through the C ABI of include/vaeb_hip.h.  There is no CPU fallback.
"""
from __future__ import annotations

import pickle

import numpy as np

from . import _lib
from . import pickle_static
from .infalg import AdaGrad, bind_updates

PARAM_NAMES_BERNOULLI = ["W3", "W4", "W5", "W1", "W2", "b3", "b4", "b5", "b1", "b2"]
PARAM_NAMES_GAUSSIAN = ["W3", "W4", "W5", "W1", "W2", "W6", "b3", "b4", "b5", "b1", "b2", "b6"]


def param_shapes(D, H, Z, continuous):
    """Reference order and shapes (VAEB.py:58-115)."""
    shp = {"W3": (D, H), "W4": (H, Z), "W5": (H, Z), "W1": (Z, H), "W2": (H, D), "W6": (H, D),
           "b3": (H,), "b4": (Z,), "b5": (Z,), "b1": (H,), "b2": (D,), "b6": (D,)}
    names = PARAM_NAMES_GAUSSIAN if continuous else PARAM_NAMES_BERNOULLI
    return [(n, shp[n]) for n in names]


def initial_params(D, H, Z, continuous):
    """VAEB.initialize_params (VAEB.py:50-115): RandomState(10) (forced, VAEB.py:148),
    std 0.01 normal weights cast to float32, zero biases; W3 and W4 are drawn twice and
    the first draws discarded (VAEB.py:58-67 duplicated at :76-85)."""
    prng = np.random.RandomState(10)
    w = lambda a, b: prng.normal(0, 0.01, (a, b)).astype(np.float32)
    w(D, H)
    w(H, Z)
    vals = {"W3": w(D, H), "W4": w(H, Z), "W5": w(H, Z), "W1": w(Z, H), "W2": w(H, D)}
    if continuous:
        vals["W6"] = w(H, D)
    out = []
    for n, s in param_shapes(D, H, Z, continuous):
        out.append(vals[n] if n in vals else np.zeros(s, np.float32))
    return out


def dtype_name(dtype):
    """The engine a dtype name selects: "float32" (aliases f32, fp32), "bf16" (bfloat16) or
    "fp16" (float16, f16, half): the 16-bit MFMA engine with bf16 or fp16 operands."""
    d = str(dtype).lower()
    if d in ("float32", "f32", "fp32"):
        return "float32"
    if d in ("bf16", "bfloat16"):
        return "bf16"
    if d in ("fp16", "float16", "f16", "half"):
        return "fp16"
    raise ValueError(f"dtype {dtype!r}: float32, bf16 or fp16")


def lib_dtype(name):
    """The library's vaeb_dtype for a dtype_name()."""
    from . import _lib
    return {"float32": _lib.DTYPE_F32, "bf16": _lib.DTYPE_BF16, "fp16": _lib.DTYPE_F16}[dtype_name(name)]


def train_rows(data):
    """The training images of a dataset in either form VAEB.load returns (VAEB.py:229-239):
    (x_train, x_valid) for Frey, or mnist.pkl.gz's ((x, y) train, valid, test) for MNIST.
    (The tuple test comes first: np.ndim of the ragged (images, labels) pair raises.)"""
    return data[0][0] if isinstance(data[0], tuple) else data[0]


class SharedParam:
    """Stand-in for a Theano shared parameter of the reference (`.name`, `.get_value()`,
    `.set_value()`, `.eval()`), backed by the device arena of the owning model."""

    def __init__(self, model, index, name, shape):
        self._m, self._i, self.name, self.shape = model, index, name, shape

    def get_value(self, borrow=False):
        return self._m._param_arrays()[self._i]

    def set_value(self, value, borrow=False):
        arrs = self._m._param_arrays()
        arrs[self._i] = np.asarray(value, np.float32).reshape(self.shape)
        self._m._ctx.set_params(np.concatenate([a.ravel() for a in arrs]))

    def eval(self):
        return self.get_value()

    def __repr__(self):
        return f"SharedParam({self.name}, {self.shape})"


def _as_array(p):
    if isinstance(p, SharedParam):
        return p.get_value()
    if hasattr(p, "get_value"):
        return np.asarray(p.get_value())
    return np.asarray(p)


class TheanoStreamEmulation:
    """Host noise emulating theano RandomStreams(seed=10) as recalled in SURVEY 8(c):
    each random op (one per L sample, VAEB.py:334-336) owns RandomState(seedgen.randint(2**30))
    and `update` and `validate` share those states.  Unverified against Theano (absent)."""

    def __init__(self, L, seed=10):
        seedgen = np.random.RandomState(seed)
        self.states = [np.random.RandomState(seedgen.randint(2 ** 30)) for _ in range(L)]

    def draw(self, rows, Z):
        return np.stack([st.normal(0.0, 1.0, size=(rows, Z)) for st in self.states]).astype(np.float32)


class VAEB:
    """Drop-in for the reference class (VAEB.py:132-133 signature).

    Extra keyword-only arguments (not in the reference): device, rng ("philox": on-device
    counter-based normals keyed by (seed, step, row); "theano": host RandomStreams
    emulation), seed, objective ("sum_prior" = VAEB.py; "mean_map" = VAEBfullbayes.py),
    use_graph, max_eval_rows; B_global / row_offset / comm for data parallelism (this rank's
    batch_size rows start at row_offset of each B_global-row global minibatch; comm = a
    (uid, rank, world) RCCL id for vaeb_comm_init, see dp.comm_setup); dtype "float32" (the
    reference's floatX, run_on_gpu.sh:2) or "bf16" (bf16 MFMA operands, fp32 master weights)."""

    def __init__(self, x_train, continuous, hidden_units, latent_size, batch_size, L, learning_rate,
                 genericEstimator, fullVariational, params=None, prng=None, sigmaInit=None, *,
                 device=0, rng="philox", seed=10, objective="sum_prior", use_graph=True, max_eval_rows=10000,
                 B_global=None, row_offset=0, fv_sample=False, inf=None, dtype="float32", comm=None):
        x_train = np.asarray(x_train, np.float32)
        self.dtype = dtype_name(dtype)
        if inf is not None:
            # optimizer plug-in (degenerate-vae/infalg.py contract): its eta is the step size
            learning_rate = inf.eta
        self.N, self.input_size = x_train.shape
        self.n_hidden_units = hidden_units
        self.n_latent = latent_size
        self.continuous = bool(continuous)
        self.learning_rate = learning_rate
        self.batch_size = batch_size
        # the reference ignores prng / sigmaInit (VAEB.py:141-149): RandomState(10), 0.01
        self.prng = np.random.RandomState(10)
        self.sigmaInit = 0.01
        self.L = L
        self.eps = 1e-6
        self.rho = 0.95
        self.fullVBSigmaInit = 1e-3
        self.genericEstimator = bool(genericEstimator)
        self.fullVariational = bool(fullVariational)
        self.objective = objective
        if self.fullVariational:
            assert params is not None
        # fv_sample (extension): full-variational with the weight-posterior sample of
        # sample_variational_params (VAEB.py:127-129) in the data term
        self.fv_sample = bool(fv_sample) and self.fullVariational
        est = _lib.EST_LA if self.genericEstimator else (
            (_lib.EST_FVS if self.fv_sample else _lib.EST_FV) if self.fullVariational else _lib.EST_LB)
        self._ctx = _lib.Context(self.input_size, hidden_units, latent_size, batch_size, L=L,
                                 decoder=_lib.DEC_GAUSSIAN if self.continuous else _lib.DEC_BERNOULLI,
                                 estimator=est,
                                 objective=_lib.OBJ_MEAN_MAP if objective == "mean_map" else _lib.OBJ_SUM_PRIOR,
                                 lr=learning_rate, adagrad_eps=self.eps, device=device, B_global=B_global,
                                 row_offset=row_offset, max_eval_rows=max_eval_rows, use_graph=use_graph,
                                 dtype=lib_dtype(self.dtype))
        self.B_global = B_global or batch_size
        self.row_offset = row_offset
        self.world, self.rank = 1, 0
        if comm is not None:
            uid, self.rank, self.world = comm
            self._ctx.comm_init(uid, self.rank, self.world)
        self._shapes = param_shapes(self.input_size, hidden_units, latent_size, self.continuous)
        if params is None:
            arrs = initial_params(self.input_size, hidden_units, latent_size, self.continuous)
        else:
            arrs = [np.asarray(_as_array(p), np.float32).reshape(s) for p, (_, s) in zip(params, self._shapes)]
        self._ctx.set_params(np.concatenate([a.ravel() for a in arrs]))
        self.params = [SharedParam(self, i, n, s) for i, (n, s) in enumerate(self._shapes)]
        # the update list of VAEB.getUpdates (VAEB.py:426-444) in the infalg.construct form,
        # bound to the fused Adagrad epilogues of the engine
        self.updates = (inf or AdaGrad(learning_rate)).construct(self, self.params)
        bind_updates(self, self.params, self.updates)
        if self.fullVariational:
            # VAEB.py:120-125: mu_theta = theta, sigma_theta = 1e-3; Adagrad state zero (:178-182)
            flat = np.concatenate([a.ravel() for a in arrs])
            self._ctx.set_fv_state(flat, np.full_like(flat, self.fullVBSigmaInit), np.zeros_like(flat),
                                   np.zeros_like(flat))
        self._ctx.set_data(x_train)
        self.rng = rng
        if rng == "theano":
            self._stream = TheanoStreamEmulation(L, seed)
            self._ctx.set_eps_mode(_lib.EPS_HOST, seed)
            self._zeta_rs = np.random.RandomState(seed + 1)   # host weight noise (fv_sample)
        else:
            self._stream = None
            self._ctx.set_eps_mode(_lib.EPS_PHILOX, seed)
        self._nb = self.N // self.B_global

    # ------------------------------------------------------------------ state helpers
    def _param_arrays(self):
        flat = self._ctx.get_params()
        out, o = [], 0
        for _, s in self._shapes:
            n = int(np.prod(s))
            out.append(flat[o:o + n].reshape(s).copy())
            o += n
        return out

    def get_param_values(self):
        return self._param_arrays()

    @property
    def full_variational_params(self):
        mu, sg, _, _ = self._ctx.get_fv_state()
        out, o = [], 0
        for _, s in self._shapes:
            n = int(np.prod(s))
            out += [mu[o:o + n].reshape(s), sg[o:o + n].reshape(s)]
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

    def _acc_slice(self, param):
        o = sum(int(np.prod(s)) for _, s in self._shapes[:param._i])
        return o, o + int(np.prod(param.shape))

    def _acc_get(self, param):
        a, b = self._acc_slice(param)
        return self._ctx.get_adagrad_state()[a:b].reshape(param.shape).copy()

    def _acc_set(self, param, value):
        a, b = self._acc_slice(param)
        flat = self._ctx.get_adagrad_state()
        flat[a:b] = value.ravel()
        self._ctx.set_adagrad_state(flat)

    # ------------------------------------------------------------------ the operators
    def update(self, index):
        """VAEB.update (VAEB.py:408-415): one SGVB/Adagrad step on rows
        [index*B, (index+1)*B); returns SGVB / batch_size."""
        if self._stream is not None:
            self._ctx.push_eps(self._stream.draw(self.batch_size, self.n_latent))
            if self.fv_sample:
                self._ctx.push_fv_noise(self._zeta_rs.standard_normal(self._ctx.P).astype(np.float32))
        return self._ctx.update(int(index))

    def update_epoch(self, batch_order):
        """All steps of `batch_order` with no per-step host sync; returns the sum of the
        per-step SGVB/B values (what train_model accumulates, VAEB.py:577-579)."""
        if self._stream is not None:
            return float(sum(self.update(int(b)) for b in batch_order))
        self._ctx.epoch_elbo()   # drop what earlier update() calls added to the accumulator
        self._ctx.update_many(np.asarray(batch_order, np.int32))
        s, n = self._ctx.epoch_elbo()
        return s

    def validate(self, x):
        """VAEB.validate (VAEB.py:418-422): forward-only SGVB sum over x (mean for the
        mean_map objective, VAEBfullbayes.py:161-165)."""
        x = np.asarray(x, np.float32)
        if self._stream is not None:
            self._ctx.push_eps(self._stream.draw(x.shape[0], self.n_latent))
        v = self._ctx.validate(x)
        return v / x.shape[0] if self.objective == "mean_map" else v

    def set_validation_data(self, x):
        """Upload x_valid once (device-resident); validate_resident() then evaluates it
        each epoch with no host copy, sharded over the ranks when data-parallel."""
        x = np.asarray(x, np.float32)
        self._nvalid = x.shape[0]
        self._ctx.set_valid_data(x)

    def validate_resident(self):
        """validate(x_valid) on the resident validation set: SGVB sum (mean for the
        mean_map objective), all-reduced over the ranks."""
        if self._stream is not None:
            self._ctx.push_eps(self._stream.draw(self._nvalid, self.n_latent))
        v = self._ctx.validate_resident()
        return v / self._nvalid if self.objective == "mean_map" else v

    def reconstruct(self, x, n_samples=0, mean=False):
        """VAEB.reconstruct (VAEB.py:267-300): the decoder output at z = mu for n_samples <= 0,
        else averaged over n_samples posterior draws z = mu + exp(lv / 2) eps (:271-291).
        The Bernoulli decoder returns those means.  The continuous decoder, as the reference,
        returns one draw N(y_mu, exp(y_log_sigma)^2 I) from numpy's global generator
        (:293-297; drawn per pixel as y_mu + exp(y_log_sigma) * np.random.standard_normal,
        the same distribution as the reference's multivariate_normal with a diagonal
        covariance, not the same stream).  mean=True (extension) returns y_mu instead.
        A 1-D x (one row, as reconstruction.py:32 passes) gives a 1-D result."""
        x = np.asarray(x, np.float32)
        one = x.ndim == 1
        x = np.atleast_2d(x)
        if n_samples > 0 and self._stream is not None:
            # one srng.normal draw per sample (VAEB.py:280), rows stacked sample-major
            self._ctx.push_eps(np.concatenate([self._stream.draw(x.shape[0], self.n_latent)
                                               for _ in range(n_samples)], axis=1))
        y, ls = self._ctx.reconstruct_full(x, max(int(n_samples), 0), log_sigma=self.continuous and not mean)
        if ls is not None:
            y = (y.astype(np.float64) + np.exp(ls.astype(np.float64)) * np.random.standard_normal(y.shape))
        return y[0] if one else y

    def decoder(self, z):
        """VAEB.decoder (VAEB.py:253-265) evaluated at given latents z [n x Z]: (mu,
        log_sigma) for the continuous decoder, y for the Bernoulli one."""
        mu, ls = self._ctx.decode(np.asarray(z, np.float32))
        return (mu, ls) if self.continuous else mu

    def freyFace(self, z):
        """The compiled `freyFace` function of freyFace.py (:173-187, 237-245): the decoder at
        z -- [mu, log_sigma] (continuous) or y (Bernoulli), float64 like the reference's
        dmatrix output."""
        out = self.decoder(z)
        if self.continuous:
            return [out[0].astype(np.float64), out[1].astype(np.float64)]
        return out.astype(np.float64)

    # ------------------------------------------------------------------ checkpoints
    def save(self, file_name):
        """VAEB.save (VAEB.py:189-203): header frames then one frame per parameter.
        Writes the 9-field header VAEB.load reads (VAEB.py:210-218); parameters are plain
        float32 ndarrays (no Theano wrapper)."""
        print('Saving model to: {0}'.format(file_name))
        with open(file_name, "wb") as f:
            # the reference-level batch size: under data parallelism self.batch_size is this
            # rank's share, B_global the minibatch a step covers
            for v in (self.n_hidden_units, self.n_latent, self.continuous, self.learning_rate, self.B_global,
                      np.random.RandomState(10), self.sigmaInit, self.L, self.genericEstimator):
                pickle.dump(v, f, protocol=2)
            for a in self._param_arrays():
                pickle.dump(a, f, protocol=2)

    def save_state(self, file_name):
        """Native checkpoint (vaeb_checkpoint_save): theta, the Adagrad accumulators, the
        Philox seed / step and the variational state -- everything a bit-identical resume
        needs, unlike the reference's .mdl (VAEB.py:189-203 keeps theta only).  With a
        data-parallel communicator every rank calls it (the sharded Adagrad state is gathered
        first); file_name None joins that gather without writing."""
        self._ctx.checkpoint_save(file_name)

    def load_state(self, file_name):
        """Resume from save_state's file (shape and estimator must match)."""
        self._ctx.checkpoint_load(file_name)

    @staticmethod
    def read_checkpoint(file_name):
        """(header, [param arrays]) of a reference or vaeb_amd .mdl file, decoded
        statically (vaeb_amd.pickle_static: nothing in the file is executed)."""
        return pickle_static.read_mdl(file_name)

    @staticmethod
    def load(file_name, data=None, **kw):
        """VAEB.load (VAEB.py:206-242): rebuild the model from a checkpoint and load the
        dataset as the reference does -- (x_train, x_valid) from freyfaces.pkl, or
        mnist.pkl.gz's ((x, y) train, valid, test) -- unless `data` is given (either form)."""
        print('Loading model form : {0}'.format(file_name))
        hdr, params = pickle_static.read_mdl(file_name)
        continuous = bool(hdr["continuous"])
        if data is None:
            from .cli import load_dataset
            data = load_dataset(continuous, splits=3 if not continuous else 2)
        x_train = train_rows(data)
        model = VAEB(x_train, continuous, int(hdr["n_hidden_units"]), int(hdr["n_latent"]), int(hdr["batch_size"]),
                     int(hdr["L"]), float(hdr["learning_rate"]), bool(hdr.get("genericEstimator", False)), False,
                     params, **kw)
        return model, data

    def close(self):
        self._ctx.close()
