"""CPU oracle for the VAEB SGVB training step -- TEST INFRASTRUCTURE ONLY.

This module is a NumPy restatement of the reference's hot path (budzianowski/VAEB,
read-only at /root/reference).  It exists to CHECK the HIP implementation; the
product path (vaeb_amd/) never imports it.  Only tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg may use it.

Pinning status ("Oracle"):
  * Adagrad rule, the -1/2*sum(theta^2) prior gradient, the SGVB/B output scaling and
    the literal full-variational dynamics are PINNED against the reference's own output
    file full_vb_res/continuous_2.trc (tests/test_oracle_pins.py).
  * degenerate-vae/logpdf.py:119-123 known-answer test is pinned (-0.0603014090604336).
  * The LB/LA per-step values cannot be compared to real Theano here (Theano and
    Python 2 are absent; VAEB.py is not valid Python 3), so beyond the pins above they
    are cross-checked by float64 torch autograd of the same objective
    (tests/test_oracle_autograd.py): "parity unpinned beyond restatement" for the
    bitwise Theano behaviour (softplus rewrite, RandomStreams seeding).

Every function cites the reference file:line it restates.
"""
from __future__ import annotations

import dataclasses
import math

import numpy as np

LOG2PI = math.log(2.0 * math.pi)

# Reference parameter order (VAEB.py:111-115).
PARAM_NAMES_BERNOULLI = ["W3", "W4", "W5", "W1", "W2", "b3", "b4", "b5", "b1", "b2"]
PARAM_NAMES_GAUSSIAN = ["W3", "W4", "W5", "W1", "W2", "W6", "b3", "b4", "b5", "b1", "b2", "b6"]


@dataclasses.dataclass
class Config:
    """Hyper-parameters of one VAEB model (VAEB.py:132-152)."""

    D: int
    H: int
    Z: int
    continuous: bool = False          # Gaussian decoder (Frey) vs Bernoulli (MNIST)
    L: int = 1                        # samples of z per datapoint (VAEB.py:143)
    estimator: str = "LB"             # "LB" (VAEB.py:332), "LA" (:315), "FV" (:349)
    objective: str = "sum_prior"      # "sum_prior" (VAEB.py:386-390) | "mean_map" (VAEBfullbayes.py:142,183)
    lr: float = 0.01                  # --learning_rate (VAEB.py:31)
    eps: float = 1e-6                 # Adagrad fudge factor (VAEB.py:144)
    fv_sigma_init: float = 1e-3       # VAEB.py:146

    @property
    def names(self):
        return PARAM_NAMES_GAUSSIAN if self.continuous else PARAM_NAMES_BERNOULLI


def param_shapes(cfg: Config):
    """Shapes in reference order (VAEB.py:58-115)."""
    D, H, Z = cfg.D, cfg.H, cfg.Z
    shp = {"W3": (D, H), "W4": (H, Z), "W5": (H, Z), "W1": (Z, H), "W2": (H, D), "W6": (H, D),
           "b3": (H,), "b4": (Z,), "b5": (Z,), "b1": (H,), "b2": (D,), "b6": (D,)}
    return [(n, shp[n]) for n in cfg.names]


def num_params(cfg: Config) -> int:
    return int(sum(np.prod(s) for _, s in param_shapes(cfg)))


def init_params(cfg: Config, dtype=np.float32):
    """VAEB.initialize_params (VAEB.py:50-115) with the forced prng=RandomState(10) and
    sigmaInit=0.01 (VAEB.py:148-149).  The reference draws W3 and W4 TWICE
    (VAEB.py:58-67 then :76-85); the first two draws are discarded.  Draws are float64
    normal(0, 0.01) cast to floatX (VAEB.py:52); biases are zeros (VAEB.py:53)."""
    prng = np.random.RandomState(10)
    sig = 0.01
    D, H, Z = cfg.D, cfg.H, cfg.Z
    draw = lambda a, b: prng.normal(0, sig, (a, b)).astype(np.float32)
    draw(D, H)  # W3 (discarded, VAEB.py:58)
    draw(H, Z)  # W4 (discarded, VAEB.py:64)
    W = {"W3": draw(D, H), "W4": draw(H, Z), "W5": draw(H, Z), "W1": draw(Z, H), "W2": draw(H, D)}
    if cfg.continuous:
        W["W6"] = draw(H, D)
    for n, s in param_shapes(cfg):
        if n.startswith("b"):
            W[n] = np.zeros(s, np.float32)
    return [W[n].astype(dtype) for n in cfg.names]


def init_params_fullbayes(cfg: Config, dtype=np.float32):
    """VAEBfullbayes.VAE.__init__ (VAEBfullbayes.py:23-73): its own RandomState(10)
    (:23), std 0.01 (:24), and each weight drawn ONCE in the order W3, W4, W5, W1, W2,
    (W6) (:34-67) -- unlike VAEB.initialize_params' duplicated W3/W4 draws; zero biases
    (:29); parameter list in the same reference order (:69-73)."""
    prng = np.random.RandomState(10)
    D, H, Z = cfg.D, cfg.H, cfg.Z
    draw = lambda a, b: prng.normal(0, 0.01, (a, b)).astype(np.float32)
    W = {"W3": draw(D, H), "W4": draw(H, Z), "W5": draw(H, Z), "W1": draw(Z, H), "W2": draw(H, D)}
    if cfg.continuous:
        W["W6"] = draw(H, D)
    for n, s in param_shapes(cfg):
        if n.startswith("b"):
            W[n] = np.zeros(s, np.float32)
    return [W[n].astype(dtype) for n in cfg.names]


def flatten(params):
    return np.concatenate([np.asarray(p).ravel() for p in params])


def unflatten(flat, cfg: Config):
    out, o = [], 0
    for _, s in param_shapes(cfg):
        n = int(np.prod(s))
        out.append(np.asarray(flat[o:o + n]).reshape(s))
        o += n
    return out


def softplus(a):
    return np.logaddexp(0.0, a).astype(a.dtype)


def sigmoid(a):
    return (1.0 / (1.0 + np.exp(-a))).astype(a.dtype)


def _unpack(params, cfg):
    d = dict(zip(cfg.names, params))
    return d


def fp16_round(a):
    """Round to the nearest IEEE binary16 (ties to even, gradual underflow), returned in a's
    dtype: the storage rounding of the 16-bit engine's fp16 instantiation
    (vaeb_amd/csrc/gemm_bf16.hpp f2bf with VAEB_H16_F16, v_cvt_f16_f32)."""
    a = np.asarray(a)
    return a.astype(np.float32).astype(np.float16).astype(a.dtype)


def fp16_round_scaled(S):
    """fp16 storage of values carried scaled by the power of two S (the fp16 engine's loss
    scale for the mean objective, engine_bf16.inc h16_scale): round(a S) / S -- the same bits
    as fp16_round for normal values, without its underflow below 6.1e-5 / S."""
    def q(a):
        a = np.asarray(a)
        return (fp16_round(a.astype(np.float64) * S) / S).astype(a.dtype)
    return q


def bf16_round(a):
    """Round to the nearest bfloat16 (ties to even), returned in a's dtype: the storage
    rounding of the bf16 engine (vaeb_amd/csrc/gemm_bf16.hpp f2bf)."""
    a = np.asarray(a)
    u = a.astype(np.float32).view(np.uint32).astype(np.uint64)
    u = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
    return u.astype(np.uint32).view(np.float32).astype(a.dtype)


def forward_backward(params, x, eps, cfg: Config, need_grad=True, q=None):
    """One SGVB evaluation and its reverse-mode gradient, restating:
      encoder VAEB.py:245-251, reparam_trick :41-47, decoder :253-265,
      posterior_log_prob :302-313, getLB :332-346 / getLA :315-330,
      criterion J = SGVB - 1/2 sum theta^2 :385-393 (objective "sum_prior"), or the
      VAEBfullbayes mean objective VAEBfullbayes.py:138-145 (objective "mean_map").
    The Bernoulli log-likelihood uses the softplus form x*a - softplus(a), which is what
    Theano FAST_RUN rewrites -binary_crossentropy(sigmoid(a), x) to.

    x: [B, D];  eps: [L, B, Z] standard normals.
    Returns dict with 'sgvb' (sum over batch, the reference's SGVB), intermediates and
    'grads' = dJ/dtheta in reference order (ascent direction, prior included).

    q: optional storage quantizer (bf16_round) applied exactly where the bf16 engine
    rounds: every GEMM operand (x, weights, h, z, hd, dA2/dA6, dA1, dMu/dLv, dA3), while
    bias gradients, log-likelihood, KL and the latent block stay in full precision.
    q=None is the plain restatement.
    """
    Q = q if q is not None else (lambda v: v)
    p = _unpack(params, cfg)
    dt = p["W3"].dtype
    x = np.asarray(x, dt)
    eps = np.asarray(eps, dt)
    B = x.shape[0]
    L = eps.shape[0]
    Z = cfg.Z
    s = dt.type(1.0 / B) if cfg.objective == "mean_map" else dt.type(1.0)
    half = dt.type(0.5)

    xq = Q(x)
    a3 = xq @ Q(p["W3"]) + p["b3"]
    h = Q(np.tanh(a3))
    mu = h @ Q(p["W4"]) + p["b4"]
    lv = h @ Q(p["W5"]) + p["b5"]
    std = np.exp(half * lv)
    z = mu[None] + std[None] * eps                    # [L, B, Z]
    zf = Q(z.reshape(L * B, Z))
    a1 = zf @ Q(p["W1"]) + p["b1"]
    hd = Q(np.tanh(a1))
    a2 = hd @ Q(p["W2"]) + p["b2"]
    xr = np.tile(xq, (L, 1))     # the bf16 engine stores the dataset itself in bf16
    y = sigmoid(a2)
    out = dict(a3=a3, h=h, mu=mu, lv=lv, z=z, hd=hd, a2=a2, y=y)
    if cfg.continuous:
        a6 = hd @ Q(p["W6"]) + p["b6"]
        r = xr - y
        # VAEB.py:306-307
        logp_rows = (dt.type(-0.5 * LOG2PI) - half * a6 - half * r * r / np.exp(a6)).sum(1)
        out["a6"] = a6
    else:
        logp_rows = (xr * a2 - softplus(a2)).sum(1)
    logp_rows = logp_rows.reshape(L, B)
    out["logp_rows"] = logp_rows
    if cfg.estimator == "LA":
        # VAEB.py:322-327
        prior = (dt.type(-0.5 * LOG2PI) - half * z * z).sum(2)
        logq = (dt.type(-0.5 * LOG2PI) - half * lv[None] - half * (z - mu[None]) ** 2 / np.exp(lv)[None]).sum(2)
        sgvb = (logp_rows + prior - logq).sum() / dt.type(L)
        out["la_rows"] = prior - logq
    else:
        # VAEB.py:343-344 (LB); FV uses the same per-row quantities (VAEB.py:358)
        kl_rows = half * (1 + lv - mu ** 2 - np.exp(lv)).sum(1)
        out["kl_rows"] = kl_rows
        sgvb = logp_rows.sum() / dt.type(L) + kl_rows.sum()
    out["sgvb"] = sgvb
    if not need_grad:
        return out

    # ---- reverse mode ----
    sl = dt.type(s / L)
    if cfg.continuous:
        e = np.exp(-a6)
        dA2 = r * e * y * (1 - y) * sl
        dA6 = (dt.type(-0.5) + half * r * r * e) * sl
    else:
        dA2 = (xr - y) * sl
    g = {}
    g["W2"] = hd.T @ Q(dA2)
    g["b2"] = dA2.sum(0)
    dHd = Q(dA2) @ Q(p["W2"]).T
    if cfg.continuous:
        g["W6"] = hd.T @ Q(dA6)
        g["b6"] = dA6.sum(0)
        dHd = dHd + Q(dA6) @ Q(p["W6"]).T
    dA1 = dHd * (1 - hd * hd)
    g["W1"] = zf.T @ Q(dA1)
    g["b1"] = dA1.sum(0)
    dZ = (Q(dA1) @ Q(p["W1"]).T).reshape(L, B, Z)
    if cfg.estimator == "LA":
        dMu = dZ.sum(0) + sl * (-z).sum(0)
        dLv = (dZ * half * std[None] * eps).sum(0) + sl * (half - half * z * std[None] * eps).sum(0)
    else:
        dMu = dZ.sum(0) - s * mu
        dLv = (dZ * half * std[None] * eps).sum(0) + s * half * (1 - np.exp(lv))
    g["W4"] = h.T @ Q(dMu)
    g["b4"] = dMu.sum(0)
    g["W5"] = h.T @ Q(dLv)
    g["b5"] = dLv.sum(0)
    dH = Q(dMu) @ Q(p["W4"]).T + Q(dLv) @ Q(p["W5"]).T
    dA3 = dH * (1 - h * h)
    g["W3"] = xq.T @ Q(dA3)
    g["b3"] = dA3.sum(0)
    out.update(dA2=dA2, dA1=dA1, dZ=dZ, dMu=dMu, dLv=dLv, dA3=dA3)
    if cfg.continuous:
        out["dA6"] = dA6
    prior_coef = dt.type(1.0) if cfg.objective == "sum_prior" else dt.type(0.0)
    out["data_grads"] = [g[n].astype(dt) for n in cfg.names]
    out["grads"] = [(g[n] - prior_coef * p[n]).astype(dt) for n in cfg.names]
    return out


def adagrad_update(params, acc, grads, cfg: Config):
    """VAEB.getUpdates (VAEB.py:426-444): acc' = acc + g^2;
    theta' = theta + lr*g/(sqrt(acc') + eps).  All updates simultaneous.
    For objective "mean_map" adds the VAEBfullbayes.py:183-184 decay -lr*eps*theta^2.
    Same rule as degenerate-vae/infalg.py:148-164 (AdaGrad.construct)."""
    new_p, new_a = [], []
    for th, a, g in zip(params, acc, grads):
        dt = th.dtype
        a2 = a + g * g
        upd = th + dt.type(cfg.lr) * g / (np.sqrt(a2) + dt.type(cfg.eps))
        if cfg.objective == "mean_map":
            upd = upd - dt.type(cfg.lr) * dt.type(cfg.eps) * th * th
        new_p.append(upd.astype(dt))
        new_a.append(a2.astype(dt))
    return new_p, new_a


def step(params, acc, x, eps, cfg: Config, q=None):
    """VAEB.update(index) (VAEB.py:408-415): returns (SGVB/B, theta', acc', aux)."""
    out = forward_backward(params, x, eps, cfg, q=q)
    B = x.shape[0]
    new_p, new_a = adagrad_update(params, acc, out["grads"], cfg)
    return out["sgvb"] / B, new_p, new_a, out


def validate(params, x, eps, cfg: Config, q=None):
    """VAEB.validate (VAEB.py:418-422): forward-only SGVB *sum* over all rows of x.
    (The mean_map variant returns the mean, VAEBfullbayes.py:161-165.)"""
    out = forward_backward(params, x, eps, cfg, need_grad=False, q=q)
    if cfg.objective == "mean_map":
        return out["sgvb"] / x.shape[0]
    return out["sgvb"]


def reconstruct(params, x, eps, cfg: Config):
    """VAEB.reconstruct (VAEB.py:267-300).  eps: None (n_samples <= 0: decoder at z = mu,
    :269-270) or [S, B, Z] standard normals, one draw per sample (:279-280); the decoder
    outputs are summed in sample order and divided by S (:277-291).  Returns the Bernoulli
    means y, or for the continuous decoder the averaged decoder mean (the reference's closing
    np.random.multivariate_normal over a [B x D] mean, :292-296, cannot run)."""
    p = _unpack(params, cfg)
    dt = p["W3"].dtype
    x = np.asarray(x, dt)
    h = np.tanh(x @ p["W3"] + p["b3"])
    mu = h @ p["W4"] + p["b4"]
    lv = h @ p["W5"] + p["b5"]

    def dec(z):
        hd = np.tanh(z @ p["W1"] + p["b1"])
        return sigmoid(hd @ p["W2"] + p["b2"])

    if eps is None:
        return dec(mu)
    eps = np.asarray(eps, dt)
    y = np.zeros((x.shape[0], cfg.D), dt)
    for s in range(eps.shape[0]):
        y = y + dec(mu + np.exp(dt.type(0.5) * lv) * eps[s])
    return y / dt.type(eps.shape[0])


def decode(params, z, cfg: Config):
    """The decoder from given latents: freyFace.py:173-187 `image(z)` (compiled as `freyFace`,
    :237-245) / VAEB.decoder (VAEB.py:253-265).  Returns (mu, log_sigma); log_sigma is None
    for the Bernoulli decoder."""
    p = _unpack(params, cfg)
    dt = p["W1"].dtype
    hd = np.tanh(np.asarray(z, dt) @ p["W1"] + p["b1"])
    mu = sigmoid(hd @ p["W2"] + p["b2"])
    return mu, (hd @ p["W6"] + p["b6"] if cfg.continuous else None)


def reconstruct_full(params, x, eps, cfg: Config):
    """VAEB.reconstruct (VAEB.py:267-291) up to its closing draw: (y_mu, y_log_sigma), each
    the decoder output at z = mu (eps None) or the mean over the S draws of eps [S, B, Z]
    (:279-290).  The reference then returns N(y_mu, exp(y_log_sigma)^2 I) (:293-297)."""
    p = _unpack(params, cfg)
    dt = p["W3"].dtype
    x = np.asarray(x, dt)
    h = np.tanh(x @ p["W3"] + p["b3"])
    mu = h @ p["W4"] + p["b4"]
    lv = h @ p["W5"] + p["b5"]
    if eps is None:
        return decode(params, mu, cfg)
    eps = np.asarray(eps, dt)
    ym, yl = 0, 0
    for s in range(eps.shape[0]):
        m, l = decode(params, mu + np.exp(dt.type(0.5) * lv) * eps[s], cfg)
        ym = ym + m
        yl = yl + (l if l is not None else 0)
    S = dt.type(eps.shape[0])
    return ym / S, (yl / S if cfg.continuous else None)


# ---------------------------------------------------------------- full variational
def fv_theta_prior(mu_list, sig_list):
    """VAEB.py:359-363: sum over params of 1/2 sum(1 + log sigma^2 - mu^2 - sigma^2)."""
    tot = 0.0
    for m, s in zip(mu_list, sig_list):
        dt = m.dtype
        tot += float((dt.type(0.5) * (1 + np.log(s * s) - m * m - s * s)).sum(dtype=np.float64))
    return tot


def fv_step(theta_fixed, vb_mu, vb_sig, acc_mu, acc_sig, x, eps, cfg: Config):
    """Literal --full_varational step (VAEB.py:349-367, 117-125, 392-393, 426-444).
    The data term uses the FIXED loaded theta (sample_variational_params is never
    called, VAEB.py:352).  The gradient reaches (mu_theta, sigma_theta) only via
    thetaPrior and the L2 term: g_mu = -2 mu, g_sigma = 1/sigma - 2 sigma.
    Returns (SGVB/B, mu', sig', acc_mu', acc_sig', sgvb_total)."""
    cfg_lb = dataclasses.replace(cfg, estimator="LB")
    out = forward_backward(theta_fixed, x, eps, cfg_lb, need_grad=False)
    B = x.shape[0]
    data = float(out["logp_rows"].sum(dtype=np.float64)) / eps.shape[0] + float(out["kl_rows"].sum(dtype=np.float64))
    tp = fv_theta_prior(vb_mu, vb_sig)
    sgvb = B * data + tp
    gm = [(-2 * m).astype(m.dtype) for m in vb_mu]
    gs = [(1 / s - 2 * s).astype(s.dtype) for s in vb_sig]
    new_mu, new_am = adagrad_update(vb_mu, acc_mu, gm, cfg)
    new_sig, new_as = adagrad_update(vb_sig, acc_sig, gs, cfg)
    return sgvb / B, new_mu, new_sig, new_am, new_as, sgvb


def fvs_step(vb_mu, vb_sig, acc_mu, acc_sig, x, eps, zeta, cfg: Config):
    """Weight-sampling full-variational step (extension, VAEB_EST_FVS): getFVBL
    (VAEB.py:349-367) with the sample that VAEB.sample_variational_params (VAEB.py:127-129)
    defines but the reference never calls, theta~ = mu + |sigma| * zeta, in the data term.
    Criterion as the literal path (VAEB.py:386-399):
        J = B (sum log p + sum KL)(theta~) + thetaPrior(mu, sigma) - 1/2 sum (mu^2 + sigma^2)
        dJ/dmu    = B G - 2 mu,   dJ/dsigma = B G zeta sign(sigma) + 1/sigma - 2 sigma,
    G = d(sum log p + sum KL)/d theta~ (the LB data gradient at theta~).
    Returns (SGVB/B, mu', sig', acc_mu', acc_sig', sgvb_total)."""
    cfg_lb = dataclasses.replace(cfg, estimator="LB")
    theta = [m + np.abs(s) * z for m, s, z in zip(vb_mu, vb_sig, zeta)]
    out = forward_backward(theta, x, eps, cfg_lb, need_grad=True)
    B = x.shape[0]
    data = float(out["logp_rows"].sum(dtype=np.float64)) / eps.shape[0] + float(out["kl_rows"].sum(dtype=np.float64))
    tp = fv_theta_prior(vb_mu, vb_sig)
    sgvb = B * data + tp
    gm = [(B * G - 2 * m).astype(m.dtype) for G, m in zip(out["data_grads"], vb_mu)]
    gs = [(B * G * z * np.sign(s) + 1 / s - 2 * s).astype(s.dtype)
          for G, z, s in zip(out["data_grads"], zeta, vb_sig)]
    new_mu, new_am = adagrad_update(vb_mu, acc_mu, gm, cfg)
    new_sig, new_as = adagrad_update(vb_sig, acc_sig, gs, cfg)
    return sgvb / B, new_mu, new_sig, new_am, new_as, sgvb


# ---------------------------------------------------------------- logpdf (degenerate-vae)
def logpdf_bernoulli(Y, P):
    """degenerate-vae/logpdf.py:85-86 (epsilon inside the log)."""
    Y = np.asarray(Y, np.float64)
    P = np.asarray(P, np.float64)
    return float(np.sum(Y * np.log(P + 1e-7) + (1 - Y) * np.log(1.0 - P + 1e-7)))


def logpdf_indep_normal(Y, mu, logs2):
    """degenerate-vae/logpdf.py:112-114."""
    return float(-0.5 * np.sum(LOG2PI + logs2 + (Y - mu) ** 2 / np.exp(logs2)))


# ---------------------------------------------------------------- RNG / data
def theano_eps_stream(seed=10):
    """Emulation of theano RandomStreams(seed=10) as recalled in SURVEY 8(c): a seed
    generator RandomState(seed) hands each random op RandomState(randint(2**30)); each
    call draws float64 normals cast to float32.  Unverified against Theano (absent);
    parity tests inject eps instead.  Returns a function (shape) -> eps for ONE op."""
    seedgen = np.random.RandomState(seed)
    st = np.random.RandomState(seedgen.randint(2 ** 30))

    def draw(shape):
        return st.normal(0.0, 1.0, size=shape).astype(np.float32)
    return draw


def batch_orders(seed, n_batches, n_epochs):
    """train_model's batch order (VAEB.py:526, 571-577): np.random.seed(seed) then one
    in-place shuffle of arange(n_batches) per epoch."""
    np.random.seed(seed)
    order = np.arange(n_batches)
    res = []
    for _ in range(n_epochs):
        np.random.shuffle(order)
        res.append(order.copy())
    return res


def synthetic_mnist(n=50000, D=784, seed=0, binary=True):
    """SURVEY 8(d) MNIST-shaped synthetic data: per-pixel probabilities p ~ Beta(0.2,1.3)
    from default_rng(1); x = (U < p) from default_rng(seed)."""
    p = np.random.default_rng(1).beta(0.2, 1.3, size=D).astype(np.float32)
    rng = np.random.default_rng(seed)
    if binary:
        return (rng.random((n, D), dtype=np.float32) < p).astype(np.float32)
    return np.clip(p + 0.1 * rng.standard_normal((n, D), dtype=np.float32), 0, 1).astype(np.float32)


def synthetic_frey(n=1965, D=560, seed=2):
    """SURVEY 8(d) Frey-shaped synthetic data: x ~ Beta(2,2)."""
    return np.random.default_rng(seed).beta(2.0, 2.0, size=(n, D)).astype(np.float32)
