"""Parity of the HIP SGVB step (libvaeb_hip.so, through the C ABI) against the CPU
oracle (oracle/vaeb_oracle.py, float64) on identical theta / acc / x / eps.

Tolerances (stated per SURVEY 8(d)):
  * ELBO (SGVB/B): relative error <= 1e-4 (observed ~1e-6)
  * data gradients: norm-wise relative error <= 1e-4 per parameter tensor
  * theta' after Adagrad: |diff| <= 1e-3 * lr for all but a 1e-4 fraction of elements
    (the first Adagrad step is ~lr*sign(g); elements with |g| ~ 1e-6 may flip), and
    never more than 2 * lr
  * forward activations: absolute error <= 1e-5
"""
import numpy as np
import pytest

from oracle import vaeb_oracle as O

pytestmark = pytest.mark.gpu

EST = {"LB": 0, "LA": 1, "FV": 2, "FVS": 3}
OBJ = {"sum_prior": 0, "mean_map": 1}


def make_ctx(cfg, B, keep_grads=True, use_graph=True, max_eval_rows=1000):
    from vaeb_amd import _lib
    return _lib.Context(cfg.D, cfg.H, cfg.Z, B, L=cfg.L, decoder=int(cfg.continuous), estimator=EST[cfg.estimator],
                        objective=OBJ[cfg.objective], lr=cfg.lr, keep_grads=keep_grads, use_graph=use_graph,
                        max_eval_rows=max_eval_rows)


def data_for(cfg, n, seed=0):
    if cfg.continuous:
        return O.synthetic_frey(n=n, D=cfg.D, seed=seed)
    return O.synthetic_mnist(n=n, D=cfg.D, seed=seed)


def rel(a, b):
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def check_theta(new, ref, lr):
    d = np.abs(new - ref)
    assert d.max() <= 2 * lr + 1e-7, d.max()
    frac = float((d > 1e-3 * lr).mean())
    assert frac <= 1e-4, frac


CASES = [
    ("mnist20", dict(D=784, H=500, Z=20), 100),
    ("odd_shapes", dict(D=37, H=19, Z=3), 13),
    ("frey2_gauss", dict(D=560, H=200, Z=2, continuous=True), 100),
    ("mnist_LA_L2", dict(D=784, H=500, Z=20, estimator="LA", L=2), 100),
    ("mnist_LB_L3_odd", dict(D=50, H=33, Z=7, L=3), 21),
    ("frey_LA", dict(D=560, H=200, Z=5, continuous=True, estimator="LA", L=2), 100),
    ("mean_map_frey10", dict(D=560, H=200, Z=10, continuous=True, objective="mean_map"), 100),
    ("mean_map_mnist", dict(D=784, H=500, Z=10, objective="mean_map"), 100),
    ("mean_map_mnist20", dict(D=784, H=500, Z=20, objective="mean_map"), 100),   # config 4 shapes
    ("wide_latent_generic", dict(D=64, H=40, Z=40, L=2), 20),
    ("wide_latent_LA", dict(D=66, H=48, Z=36, estimator="LA"), 30),
    ("gauss_odd_D", dict(D=45, H=30, Z=6, continuous=True), 17),
    ("batch1", dict(D=784, H=500, Z=20), 1),                 # a single-row minibatch
    ("latent1_LA_L2", dict(D=30, H=17, Z=1, estimator="LA", L=2), 5),
    ("mnist_B1024", dict(D=784, H=500, Z=20), 1024),         # fp32 engine at a large batch
    ("gauss_B333", dict(D=560, H=200, Z=2, continuous=True), 333),
    # atomic latent hand-offs (fan-in <= 16) with two fx slots per thread (Z > 16)
    ("latent24_atomic_L2", dict(D=784, H=128, Z=24, L=2), 100),
    ("latent28_atomic_LA", dict(D=200, H=96, Z=28, estimator="LA", L=2), 50),
]


@pytest.mark.parametrize("name,kw,B", CASES, ids=[c[0] for c in CASES])
def test_single_step_parity(name, kw, B):
    cfg = O.Config(**kw)
    x = data_for(cfg, 4 * B)
    params = O.init_params(cfg)
    rng = np.random.default_rng(3)
    # non-zero biases so every bias path is exercised
    params = [p if p.ndim == 2 else (0.01 * rng.standard_normal(p.shape)).astype(np.float32) for p in params]
    acc = [np.zeros_like(p) for p in params]
    eps = rng.standard_normal((cfg.L, B, cfg.Z)).astype(np.float32)
    idx = 2
    xb = x[idx * B:(idx + 1) * B]

    ctx = make_ctx(cfg, B)
    ctx.set_data(x)
    ctx.set_params(O.flatten(params))
    ctx.set_adagrad_state(O.flatten(acc))
    ctx.set_eps_mode(1)
    ctx.push_eps(eps)
    elbo = ctx.update(idx)

    p64 = [p.astype(np.float64) for p in params]
    a64 = [a.astype(np.float64) for a in acc]
    ref_elbo, ref_p, ref_a, aux = O.step(p64, a64, xb.astype(np.float64), eps.astype(np.float64), cfg)
    assert abs(elbo - ref_elbo) <= 1e-4 * abs(ref_elbo), (elbo, ref_elbo)

    # forward activations
    h = ctx.activation("h", ((B + 15) // 16 * 16) * cfg.H).reshape(-1, cfg.H)[:B]
    assert np.abs(h - aux["h"]).max() <= 1e-5
    mu = ctx.activation("mu", ((B + 15) // 16 * 16) * cfg.Z).reshape(-1, cfg.Z)[:B]
    assert np.abs(mu - aux["mu"]).max() <= 1e-5

    g = ctx.get_grads()
    for (n, s), gg, rr in zip(O.param_shapes(cfg), O.unflatten(g, cfg), aux["data_grads"]):
        assert rel(gg.reshape(s), rr) <= 1e-4, (n, rel(gg.reshape(s), rr))

    newp = ctx.get_params()
    check_theta(newp, O.flatten(ref_p), cfg.lr)
    newa = ctx.get_adagrad_state()
    assert rel(newa, O.flatten(ref_a)) <= 1e-4


def test_trajectory_50_steps_mnist():
    """50 consecutive steps (graph replay, device-resident batch order) track the oracle."""
    cfg = O.Config(D=784, H=500, Z=20)
    B = 100
    x = data_for(cfg, 1000)
    params = O.init_params(cfg)
    acc = [np.zeros_like(p) for p in params]
    ctx = make_ctx(cfg, B, keep_grads=False)
    ctx.set_data(x)
    ctx.set_params(O.flatten(params))
    ctx.set_eps_mode(1)
    rng = np.random.default_rng(11)
    order = rng.permutation(10)
    p, a = [q.astype(np.float64) for q in params], [q.astype(np.float64) for q in acc]
    elbos, refs = [], []
    for t in range(50):
        b = int(order[t % 10])
        eps = rng.standard_normal((1, B, cfg.Z)).astype(np.float32)
        ctx.push_eps(eps)
        elbos.append(ctx.update(b))
        e, p, a, _ = O.step(p, a, x[b * B:(b + 1) * B].astype(np.float64), eps.astype(np.float64), cfg)
        refs.append(e)
    elbos, refs = np.array(elbos), np.array(refs)
    assert np.all(np.abs(elbos - refs) <= 1e-3 * np.abs(refs)), np.abs(elbos - refs).max()
    newp = ctx.get_params()
    assert np.abs(newp - O.flatten(p)).max() <= 5e-3


@pytest.mark.parametrize("continuous", [False, True])
def test_validate_matches_oracle(continuous):
    cfg = O.Config(D=560, H=200, Z=2, continuous=True) if continuous else O.Config(D=784, H=500, Z=20)
    n = 2500
    x = data_for(cfg, n, seed=5)
    params = O.init_params(cfg)
    rng = np.random.default_rng(2)
    eps = rng.standard_normal((1, n, cfg.Z)).astype(np.float32)
    ctx = make_ctx(cfg, 100, max_eval_rows=1000)  # 3 device chunks
    ctx.set_data(x[:1000])
    ctx.set_params(O.flatten(params))
    ctx.set_eps_mode(1)
    ctx.push_eps(eps)
    v = ctx.validate(x)
    ref = O.validate([q.astype(np.float64) for q in params], x.astype(np.float64), eps.astype(np.float64), cfg)
    assert abs(v - ref) <= 1e-4 * abs(ref), (v, ref)


def test_reconstruct_matches_oracle():
    cfg = O.Config(D=784, H=500, Z=20)
    x = data_for(cfg, 300, seed=9)
    params = O.init_params(cfg)
    ctx = make_ctx(cfg, 100)
    ctx.set_data(x)
    ctx.set_params(O.flatten(params))
    y = ctx.reconstruct(x)
    out = O.forward_backward([q.astype(np.float64) for q in params], x.astype(np.float64),
                             np.zeros((1, 300, cfg.Z)), cfg, need_grad=False)
    assert np.abs(y - out["y"]).max() <= 1e-5


@pytest.mark.parametrize("continuous", [False, True])
def test_reconstruct_sampled_matches_oracle(continuous):
    """VAEB.reconstruct(x, n_samples > 0) (VAEB.py:271-291) with host-injected eps: the
    decoder output averaged over the samples, |diff| <= 1e-5."""
    cfg = O.Config(D=560, H=200, Z=2, continuous=True) if continuous else O.Config(D=784, H=500, Z=20)
    x = data_for(cfg, 250, seed=11)
    params = O.init_params(cfg)
    rng = np.random.default_rng(12)
    S = 3
    eps = rng.standard_normal((S, 250, cfg.Z)).astype(np.float32)
    ctx = make_ctx(cfg, 100, max_eval_rows=128)   # two device chunks
    ctx.set_data(x)
    ctx.set_params(O.flatten(params))
    from vaeb_amd import _lib
    ctx.set_eps_mode(_lib.EPS_HOST)
    ctx.push_eps(eps.reshape(1, S * 250, cfg.Z))
    y = ctx.reconstruct_sampled(x, S)
    ref = O.reconstruct([q.astype(np.float64) for q in params], x.astype(np.float64), eps.astype(np.float64), cfg)
    assert np.abs(y - ref).max() <= 1e-5
    # n_samples <= 0 is the z = mu branch
    y0 = ctx.reconstruct_sampled(x, 0)
    assert np.abs(y0 - O.reconstruct([q.astype(np.float64) for q in params], x.astype(np.float64), None, cfg)).max() <= 1e-5


def test_reconstruct_sampled_philox():
    """Device-drawn samples: deterministic, distinct from z = mu, and converging to the
    posterior-mean reconstruction as S grows (statistical)."""
    cfg = O.Config(D=784, H=500, Z=20)
    x = data_for(cfg, 100, seed=13)
    params = O.init_params(cfg)
    ctx = make_ctx(cfg, 100)
    ctx.set_data(x)
    ctx.set_params(O.flatten(params))
    y1 = ctx.reconstruct_sampled(x, 4)
    y2 = ctx.reconstruct_sampled(x, 4)
    assert np.array_equal(y1, y2)
    assert np.abs(y1 - ctx.reconstruct(x)).max() > 0
    assert np.all((y1 > 0) & (y1 < 1))


def test_fv_literal_step():
    cfg = O.Config(D=560, H=200, Z=2, continuous=True, estimator="FV")
    B = 100
    x = data_for(cfg, 1500)
    theta = O.init_params(cfg)
    rng = np.random.default_rng(4)
    theta = [(t + 0.05 * rng.standard_normal(t.shape)).astype(np.float32) for t in theta]
    mu = [t.copy() for t in theta]
    sig = [np.full_like(t, 1e-3) for t in theta]
    am = [np.zeros_like(t) for t in theta]
    as_ = [np.zeros_like(t) for t in theta]
    ctx = make_ctx(cfg, B)
    ctx.set_data(x)
    ctx.set_params(O.flatten(theta))
    ctx.set_fv_state(O.flatten(mu), O.flatten(sig), O.flatten(am), O.flatten(as_))
    ctx.set_eps_mode(1)
    m64, s64 = [q.astype(np.float64) for q in mu], [q.astype(np.float64) for q in sig]
    am64, as64 = [q.astype(np.float64) for q in am], [q.astype(np.float64) for q in as_]
    t64 = [q.astype(np.float64) for q in theta]
    for t in range(3):
        eps = rng.standard_normal((1, B, cfg.Z)).astype(np.float32)
        ctx.push_eps(eps)
        e = ctx.update(t)
        ref, m64, s64, am64, as64, _ = O.fv_step(t64, m64, s64, am64, as64, x[t * B:(t + 1) * B].astype(np.float64),
                                                 eps.astype(np.float64), cfg)
        assert abs(e - ref) <= 1e-4 * abs(ref), (t, e, ref)
    gm, gs, gam, gas = ctx.get_fv_state()
    assert np.abs(gm - O.flatten(m64)).max() <= 1e-6
    assert np.abs(gs - O.flatten(s64)).max() <= 1e-7
    # theta itself is never updated on the literal FV path (SURVEY 8(c) pin 2)
    assert np.array_equal(ctx.get_params(), O.flatten(theta))


@pytest.mark.parametrize("continuous", [False, True])
def test_fv_weight_sampling_step(continuous):
    """VAEB_EST_FVS (extension): theta~ = mu + |sigma| zeta with host-injected zeta and eps,
    3 steps against oracle.fvs_step (float64).  ELBO relative <= 1e-4; mu', sigma' within
    1e-3 lr but for a 1e-3 fraction (the first Adagrad steps are ~lr sign(g)); the loaded
    theta is never written."""
    cfg = (O.Config(D=560, H=200, Z=2, continuous=True, estimator="FVS") if continuous
           else O.Config(D=784, H=500, Z=20, estimator="FVS"))
    B = 100
    x = data_for(cfg, 500)
    rng = np.random.default_rng(21)
    theta = [(t + 0.05 * rng.standard_normal(t.shape)).astype(np.float32) for t in O.init_params(cfg)]
    mu = [t.copy() for t in theta]
    sig = [np.full_like(t, 1e-3) for t in theta]
    am = [np.zeros_like(t) for t in theta]
    as_ = [np.zeros_like(t) for t in theta]
    ctx = make_ctx(cfg, B)
    ctx.set_data(x)
    ctx.set_params(O.flatten(theta))
    ctx.set_fv_state(O.flatten(mu), O.flatten(sig), O.flatten(am), O.flatten(as_))
    ctx.set_eps_mode(1)
    m64, s64 = [q.astype(np.float64) for q in mu], [q.astype(np.float64) for q in sig]
    am64, as64 = [q.astype(np.float64) for q in am], [q.astype(np.float64) for q in as_]
    for t in range(3):
        eps = rng.standard_normal((1, B, cfg.Z)).astype(np.float32)
        zeta = [rng.standard_normal(q.shape).astype(np.float32) for q in theta]
        ctx.push_eps(eps)
        ctx.push_fv_noise(O.flatten(zeta))
        e = ctx.update(t)
        ref, m64, s64, am64, as64, _ = O.fvs_step(m64, s64, am64, as64, x[t * B:(t + 1) * B].astype(np.float64),
                                                  eps.astype(np.float64), [z.astype(np.float64) for z in zeta], cfg)
        assert abs(e - ref) <= 1e-4 * abs(ref), (t, e, ref)
    gm, gs, gam, gas = ctx.get_fv_state()
    # the B-scaled data gradient (B G) makes more elements sit near g = 0, where one
    # fp32-rounding-sized difference flips a ~lr sign(g) Adagrad step: a 1e-3 fraction
    # may differ by up to 2 lr; the updates as a whole agree norm-wise to 1e-2
    for got, ref, start in ((gm, O.flatten(m64), O.flatten(mu)), (gs, O.flatten(s64), O.flatten(sig))):
        d = np.abs(got - ref)
        assert d.max() <= 2 * cfg.lr + 1e-7, d.max()
        assert float((d > 1e-3 * cfg.lr).mean()) <= 1e-3
        assert rel(got - start, ref - start) <= 1e-2
    assert np.array_equal(ctx.get_params(), O.flatten(theta))
    # validate evaluates the data term at mu_theta and adds thetaPrior (as the literal path)
    xv = x[:200]
    epsv = rng.standard_normal((1, 200, cfg.Z)).astype(np.float32)
    ctx.push_eps(epsv)
    v = ctx.validate(xv)
    cfg_lb = O.Config(**{**cfg.__dict__, "estimator": "LB"})
    mu_now = O.unflatten(gm.astype(np.float64), cfg)
    data = O.forward_backward(mu_now, xv.astype(np.float64), epsv.astype(np.float64), cfg_lb, need_grad=False)["sgvb"]
    ref_v = 200 * data + O.fv_theta_prior(mu_now, O.unflatten(gs.astype(np.float64), cfg))
    assert abs(v - ref_v) <= 1e-4 * abs(ref_v), (v, ref_v)
    ctx.close()


def test_fv_weight_sampling_philox_graph_matches_eager():
    """VAEB_EST_FVS in Philox mode: a graph-replayed sequence draws the weight sample once
    and then reads the one each fvs_update wrote for the next step (zeta(step + 1)); eager
    steps draw it every step.  The two must agree bit for bit over 40 steps (one 32-step
    replay plus single-step graphs), and the literal FV path likewise."""
    for est in ("FVS", "FV"):
        cfg = O.Config(D=784, H=500, Z=20, estimator=est)
        x = data_for(cfg, 1000)
        theta = O.init_params(cfg)
        order = np.random.default_rng(4).integers(0, 10, 40).astype(np.int32)
        outs = []
        for use_graph in (True, False):
            ctx = make_ctx(cfg, 100, keep_grads=False, use_graph=use_graph)
            ctx.set_data(x)
            ctx.set_params(O.flatten(theta))
            t = O.flatten(theta)
            ctx.set_fv_state(t, np.full_like(t, 1e-3), np.zeros_like(t), np.zeros_like(t))
            ctx.set_eps_mode(0, 10)
            ctx.set_step(0)
            ctx.update_many(order)
            outs.append((ctx.epoch_elbo(), ctx.get_fv_state()))
            ctx.close()
        assert outs[0][0] == outs[1][0], (est, outs[0][0], outs[1][0])
        for a, b in zip(outs[0][1], outs[1][1]):
            assert np.array_equal(a, b), est


def test_philox_eps_is_standard_normal_and_deterministic():
    cfg = O.Config(D=784, H=500, Z=20)
    x = data_for(cfg, 1000)
    ctx = make_ctx(cfg, 100)
    ctx.set_data(x)
    ctx.set_params(O.flatten(O.init_params(cfg)))
    ctx.set_eps_mode(0, seed=10)
    ctx.set_step(0)
    ctx.update(0)
    e1 = ctx.activation("eps", 112 * 20).reshape(112, 20)[:100]
    ctx.set_step(0)
    ctx.set_params(O.flatten(O.init_params(cfg)))
    ctx.update(0)
    e2 = ctx.activation("eps", 112 * 20).reshape(112, 20)[:100]
    assert np.array_equal(e1, e2)
    ctx.update(0)
    e3 = ctx.activation("eps", 112 * 20).reshape(112, 20)[:100]
    assert not np.array_equal(e1, e3)
    big = []
    for _ in range(20):
        ctx.update(1)
        big.append(ctx.activation("eps", 112 * 20).reshape(112, 20)[:100].ravel())
    big = np.concatenate(big)
    assert abs(big.mean()) < 0.02 and abs(big.std() - 1) < 0.02


def test_epoch_throughput_mode_matches_sync_mode():
    """update_many (graph replay, no host sync) == per-step update (same Philox noise)."""
    cfg = O.Config(D=784, H=500, Z=20)
    x = data_for(cfg, 5000)
    order = np.random.default_rng(0).permutation(50).astype(np.int32)
    res = []
    for mode in ("sync", "many"):
        ctx = make_ctx(cfg, 100, keep_grads=False)
        ctx.set_data(x)
        ctx.set_params(O.flatten(O.init_params(cfg)))
        ctx.set_eps_mode(0, seed=10)
        ctx.set_step(0)
        if mode == "sync":
            tot = sum(ctx.update(int(b)) for b in order)
        else:
            ctx.update_many(order)
            tot, n = ctx.epoch_elbo()
            assert n == len(order)
        res.append((tot, ctx.get_params()))
    assert abs(res[0][0] - res[1][0]) <= 1e-5 * abs(res[0][0])
    assert np.array_equal(res[0][1], res[1][1])


def test_update_many_call_forms_match_per_step_updates():
    """Every form an update_many call takes (vaeb_hip.hip vaeb_update_many / run_steps): one step
    (order upload + a graph from arena 0), two and twenty steps (the eager first step with the
    order upload launched behind its first kernel, then ONE graph from arena 1), 33 steps (a
    32-step graph + the remainder), 961 steps (above the kernel-argument order cap: the pinned
    staging copy ahead of the eager step), calls starting from either arena -- against the same
    minibatches as per-step synchronous updates: theta, Adagrad state and the epoch ELBO bit for
    bit (same Philox noise)."""
    cfg = O.Config(D=784, H=64, Z=8)
    B = 16
    x = data_for(cfg, 64 * B)
    rng = np.random.default_rng(3)
    calls = [rng.integers(0, 64, n).astype(np.int32) for n in (1, 2, 20, 1, 33, 961, 3)]
    res = []
    for mode in ("sync", "many"):
        ctx = make_ctx(cfg, B, keep_grads=False, max_eval_rows=B)
        ctx.set_data(x)
        ctx.set_params(O.flatten(O.init_params(cfg)))
        ctx.set_eps_mode(0, seed=5)
        ctx.set_step(0)
        if mode == "sync":
            tot = sum(ctx.update(int(b)) for o in calls for b in o)
        else:
            for o in calls:
                ctx.update_many(o)
            tot, n = ctx.epoch_elbo()
            assert n == sum(len(o) for o in calls)
        res.append((tot, ctx.get_params(), ctx.get_adagrad_state()))
        ctx.close()
    assert abs(res[0][0] - res[1][0]) <= 1e-6 * abs(res[0][0])
    assert np.array_equal(res[0][1], res[1][1])
    assert np.array_equal(res[0][2], res[1][2])


@pytest.mark.parametrize("kw", [dict(D=560, H=200, Z=2, continuous=True), dict(D=784, H=128, Z=24, L=2),
                                dict(D=784, H=500, Z=20)], ids=["frey2", "latent24_L2", "mnist20"])
def test_atomic_and_slab_handoffs_agree(kw, monkeypatch):
    """Every fp32 step form a switch can select, on the same 6 Philox steps: the default
    (VAEB_ATOMIC_HO=1: counted fixed-point atomics up to fan-in 16, slabs above), slabs +
    ticket + reducer everywhere (=0), the encoder slabs summed by the decoder launch
    (VAEB_ENC_RED=1), the unfolded latent backward (VAEB_FOLD_BWD=0: the P67 launches), the
    slab-form latent backward finished in the dhd launch (VAEB_BWD_DEFER=0) instead of the last
    launch, each step's dW2 in its own dhd launch (VAEB_DW2_DEFER=0) instead of the next
    encoder's.  (The measured-slower forms of rounds 3-5 -- one decoder column tile, 512-thread
    encoders, fixed-point encoder sums, the two-tile dhd launch -- were removed in round 6.)
    They sum the same partials in different arithmetic (exact integer vs ordered fp32), so
    they agree to rounding, and each is bitwise deterministic (graph == eager)."""
    from vaeb_amd import _lib
    cfg = O.Config(**kw)
    B = 100
    x = data_for(cfg, 8 * B)
    order = np.array([3, 1, 4, 1, 5, 7], np.int32)
    out = {}
    # "decred": VAEB_ENC_RED=1, the encoder's slabs summed by every decoder workgroup;
    # "ticket": VAEB_BWD_DEFER=0, the slab-form latent backward finished by the dhd launch's last
    # arriver (default 1: by reducer workgroups of the last launch, kernels_aux.hpp LatRed)
    # "dw2now": VAEB_DW2_DEFER=0, each step's dW2 (| dW6) in its own dhd launch (default 1: in the
    # next step's encoder launch, the last one flushed by get_params)
    # (ATOMIC_HO, ENC_RED, FOLD_BWD, BWD_DEFER, DW2_DEFER)
    modes = {"atomic": ("1", "0", "1", "1", "1"), "slab": ("0", "0", "1", "1", "1"),
             "decred": ("1", "1", "1", "1", "1"), "unfolded": ("1", "0", "0", "1", "1"),
             "ticket": ("0", "0", "1", "0", "1"), "dw2now": ("1", "0", "1", "1", "0")}
    for mode in modes:
        for use_graph in (True, False):
            for var, v in zip(("VAEB_ATOMIC_HO", "VAEB_ENC_RED", "VAEB_FOLD_BWD", "VAEB_BWD_DEFER", "VAEB_DW2_DEFER"),
                              modes[mode]):
                monkeypatch.setenv(var, v)
            ctx = _lib.Context(cfg.D, cfg.H, cfg.Z, B, L=cfg.L,
                               decoder=_lib.DEC_GAUSSIAN if cfg.continuous else _lib.DEC_BERNOULLI,
                               max_eval_rows=B, use_graph=use_graph)
            ctx.set_data(x)
            ctx.set_params(O.flatten(O.init_params(cfg)))
            ctx.set_eps_mode(_lib.EPS_PHILOX, 10)
            ctx.set_step(0)
            ctx.update_many(order)
            s_, n_ = ctx.epoch_elbo()
            out[mode, use_graph] = (s_ / n_, ctx.get_params())
            ctx.close()
    for mode in modes:
        assert out[mode, True][0] == out[mode, False][0]
        assert np.array_equal(out[mode, True][1], out[mode, False][1])
    es = out["slab", True][0]
    frac = {}
    for mode in ("atomic", "decred", "unfolded", "ticket", "dw2now"):
        ea = out[mode, True][0]
        assert abs(ea - es) <= 1e-5 * abs(es), (mode, ea, es)
        d = np.abs(out[mode, True][1] - out["slab", True][1])
        assert d.max() <= 2 * len(order) * cfg.lr, mode    # a ~lr sign(g) step may flip where |g| ~ 1e-7
        frac[mode] = float((d > 1e-3 * cfg.lr).mean())
    # Parameters whose gradient is a cancellation-dominated sum (|g| near rounding of its terms)
    # take Adagrad steps that follow that rounding (a different K split of the encoder moved
    # ~0.13 % of MNIST's parameters by more than 1e-3 lr).
    assert max(frac.values()) <= 2e-3, frac


@pytest.mark.parametrize("kw", [dict(D=784, H=500, Z=20), dict(D=560, H=200, Z=2, continuous=True)],
                         ids=["mnist20", "frey2"])
def test_deferred_dw2_is_bitwise_the_same_step(kw, monkeypatch):
    """The deferred dW2 (step t's dW2 | dW6 + Adagrad in step t+1's encoder launch, the last
    one flushed when the host reads the state) runs the same tiles with the same K split as
    the in-step form (VAEB_DW2_DEFER=0): parameters, Adagrad state and ELBO bit for bit, with
    host reads, a validation and a checkpoint round trip between calls, the synchronous
    update() among them, and graph replay as well as eager steps."""
    from vaeb_amd import _lib
    cfg = O.Config(**kw)
    x = data_for(cfg, 800)
    res = {}
    for defer in ("1", "0"):
        for use_graph in (True, False):
            monkeypatch.setenv("VAEB_DW2_DEFER", defer)
            ctx = _lib.Context(cfg.D, cfg.H, cfg.Z, 100, decoder=int(cfg.continuous), max_eval_rows=200,
                               use_graph=use_graph)
            ctx.set_data(x)
            ctx.set_params(O.flatten(O.init_params(cfg)))
            ctx.set_eps_mode(_lib.EPS_PHILOX, 10)
            out = []
            ctx.update_many(np.array([3, 1, 4, 1, 5], np.int32))
            out.append(ctx.get_params())                       # flush
            out.append(ctx.update(2))                          # sync step after a flush
            out.append(ctx.update(6))                          # sync step with a pending dW2
            out.append(ctx.validate(x[:200]))                  # flush inside the evaluation
            ctx.update_many(np.array([0, 7, 2], np.int32))
            ckpt = f"/tmp/vaeb_dw2_{defer}_{int(use_graph)}.ckpt"
            ctx.checkpoint_save(ckpt)
            ctx.update_many(np.array([5, 5], np.int32))
            out.append(ctx.get_params())
            ctx.checkpoint_load(ckpt)                          # the pending dW2 must not land on it
            ctx.update_many(np.array([5, 5], np.int32))
            out.append(ctx.get_params())
            out.append(ctx.get_adagrad_state())
            out.append(ctx.epoch_elbo()[0])
            ctx.close()
            res[defer, use_graph] = out
    ref = res["0", True]
    for key, out in res.items():
        for a, b in zip(out, ref):
            assert np.array_equal(np.asarray(a), np.asarray(b)), key
    assert np.array_equal(ref[4], ref[5])   # resume: the same two steps from the checkpoint


def test_deferred_dw2_pending_after_a_replayed_single_step():
    """a one-step update_many / update_async after a flush is a graph REPLAY with
    no eager first step; the replayed step leaves its dW2 pending, so the next host read
    (get_params, the Adagrad state, a validation, a checkpoint) must flush it.  The sequence
    the advisor named -- update_many(order), get_params, update_async(i), get_params /
    validate -- and single-step epochs between evaluations, bit for bit against the in-step
    dW2 (VAEB_DW2_DEFER=0)."""
    import os
    from vaeb_amd import _lib
    cfg = O.Config(D=784, H=500, Z=20)
    x = data_for(cfg, 800)
    res = {}
    # (defer, graph): the deferral against the in-step dW2, and replayed against eager steps
    for key in (("1", True), ("0", True), ("1", False)):
        os.environ["VAEB_DW2_DEFER"] = key[0]
        try:
            ctx = _lib.Context(cfg.D, cfg.H, cfg.Z, 100, max_eval_rows=200, use_graph=key[1])
        finally:
            del os.environ["VAEB_DW2_DEFER"]
        ctx.set_data(x)
        ctx.set_params(O.flatten(O.init_params(cfg)))
        ctx.set_eps_mode(_lib.EPS_PHILOX, 10)
        out = []
        ctx.update_many(np.array([3, 1, 4], np.int32))      # captures the graphs, replays
        out.append(ctx.get_params())                        # flush
        ctx.update_async(2)                                 # one replayed step, no eager step
        out.append(ctx.get_params())                        # must include that step's dW2
        out.append(ctx.get_adagrad_state())
        ctx.update_many(np.array([6], np.int32))            # a one-minibatch epoch
        out.append(ctx.validate(x[:200]))                   # the evaluation flushes first
        ctx.update_many(np.array([5], np.int32))
        out.append(ctx.validate(x[200:400]))
        ctx.update_many(np.array([0, 7], np.int32))         # training after the evaluations
        out.append(ctx.get_params())
        out.append(ctx.get_adagrad_state())
        out.append(ctx.epoch_elbo()[0])
        ctx.close()
        res[key] = out
    for k1, k2 in ((("1", True), ("0", True)), (("1", True), ("1", False))):
        for i, (a, b) in enumerate(zip(res[k1], res[k2])):
            assert np.array_equal(np.asarray(a), np.asarray(b)), (k1, i)


def test_fixed_point_handoff_overflow_is_reported_not_silent():
    """The counted fixed-point hand-off (latent.hpp fx_inc) at Frey 560-200-2 (fan-in 13, the
    atomic form): an encoder partial beyond its range -- here every W4 entry 1e3, so the mu
    partials reach ~1e4 * 16 hidden units -- or a NaN weight poisons the latent elements
    instead of wrapping into the count field.  The step reports VAEB_ERR_NUMERIC with NaN
    values (as the slab form's NaN propagation would), and a context restored to sane
    parameters steps cleanly again (the accumulators were reset by their completers)."""
    from vaeb_amd import _lib
    cfg = O.Config(D=560, H=200, Z=2, continuous=True)
    x = O.synthetic_frey(n=300)
    theta0 = O.flatten(O.init_params(cfg))
    ctx = _lib.Context(560, 200, 2, 100, decoder=_lib.DEC_GAUSSIAN, max_eval_rows=100)
    ctx.set_data(x)
    ctx.set_params(theta0)
    ctx.set_eps_mode(_lib.EPS_PHILOX, 10)
    good = ctx.update(0)
    assert np.isfinite(good)
    sl = O.unflatten(np.arange(theta0.size), cfg)
    for poison in ("huge", "nan"):
        bad = theta0.copy()
        bad[sl[0].ravel()] = 1.0                 # W3: h saturates at +-1
        bad[sl[1].ravel()] = 1e4 if poison == "huge" else np.nan   # W4: mu partials ~ 1e4 x 16 > 2^17
        ctx.set_params(bad)
        with pytest.raises(_lib.VaebError, match="fixed-point"):
            ctx.update(1)
        assert np.isnan(ctx.activation("mu", 100 * 2)).any()
        # the asynchronous form reports at vaeb_epoch_elbo
        ctx.set_params(bad)
        ctx.update_many(np.array([1, 2], np.int32))
        with pytest.raises(_lib.VaebError, match="fixed-point"):
            ctx.epoch_elbo()
        ctx.set_params(theta0)
        ctx.set_adagrad_state(np.zeros_like(theta0))   # the poisoned steps' NaN gradients reached it
        v = ctx.update(0)
        assert np.isfinite(v) and abs(v - good) < 0.05 * abs(good)
        assert ctx.epoch_elbo()[1] >= 1
    # the BACKWARD hand-off alone (its guard word is blk[kBlkFxErr] too, not a
    # padding word of the forward accumulators): encoder weights sane, the decoder's
    # log-sigma weights W6 NaN or huge (1e4: dA6 ~ (x - mu)^2 exp(-2 log sigma) explodes),
    # so only the dZ partials leave the range
    for poison in ("w6_nan", "w6_huge"):
        bad = theta0.copy()
        bad[sl[5].ravel()] = np.nan if poison == "w6_nan" else 1e4
        ctx.set_params(bad)
        with pytest.raises(_lib.VaebError, match="fixed-point"):
            ctx.update(1)
        assert np.all(np.isfinite(ctx.activation("mu", 100 * 2)))   # the forward hand-off stayed in range
        ctx.set_params(theta0)
        ctx.set_adagrad_state(np.zeros_like(theta0))
        v = ctx.update(0)
        assert np.isfinite(v) and abs(v - good) < 0.05 * abs(good)
    ctx.close()


def test_update_after_async_steps_returns_its_own_value():
    """vaeb_update reads the mapped result slot the step's last kernel writes; steps
    still queued from update_many / update_async would write it too.  update(j) right after
    update_async(i) must return update(j)'s own value, as a fully synchronised run does."""
    from vaeb_amd import _lib
    cfg = O.Config(D=784, H=500, Z=20)
    x = O.synthetic_mnist(n=800)
    theta0 = O.flatten(O.init_params(cfg))

    def run(sync):
        ctx = _lib.Context(784, 500, 20, 100, max_eval_rows=100)
        ctx.set_data(x)
        ctx.set_params(theta0)
        ctx.set_eps_mode(_lib.EPS_PHILOX, 10)
        out = []
        for i in range(3):
            ctx.update_async(i)
            ctx.update_many(np.array([3, 4, 5], np.int32))
            if sync:
                ctx.synchronize()
            out.append(ctx.update(6 + i % 2))
        ctx.epoch_elbo()
        ctx.close()
        return out

    assert run(False) == run(True)
