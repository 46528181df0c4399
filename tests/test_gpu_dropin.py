"""GPU tests of the round-2 drop-in pieces, all through the C ABI:

* data-parallel row offset: a rank's minibatch rows are rows [b*B_global + row_offset, +B)
  of the global minibatch b (the fp32 engine once read the first B rows on every rank);
* graph replay of any step count (32-step graphs + power-of-two tails) == eager launches;
* VAEBfullbayes.VAE (VAEBfullbayes.py:13-201): single-draw init, mean objective, MAP term,
  mean validate -- against the oracle at MNIST 784-500-20 (BASELINE config 4's named path);
* the native checkpoint: save, resume in a fresh context, and continue bit-identically;
* the device-resident validation set == the host-copy validate, and == the oracle;
* the literal FV step at MNIST 784-500-20 (config 4 shapes) against the oracle.
"""
import numpy as np
import pytest

from oracle import vaeb_oracle as O

pytestmark = pytest.mark.gpu


def rel(a, b):
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def check_theta(new, ref, lr, frac=1e-4):
    d = np.abs(new - ref)
    assert d.max() <= 2 * lr + 1e-7, d.max()
    assert float((d > 1e-3 * lr).mean()) <= frac


@pytest.mark.parametrize("with_comm", [False, True])
def test_row_offset_selects_this_ranks_rows(with_comm):
    """World-1 context playing rank 1 of 2: B = 50 of a 100-row global minibatch, rows
    [b*100 + 50, b*100 + 100).  ELBO (= SGVB / B_global), data gradients and theta' match
    the oracle's step on exactly those rows."""
    from vaeb_amd import _lib
    cfg = O.Config(D=784, H=500, Z=20)
    B, Bg, off = 50, 100, 50
    x = O.synthetic_mnist(n=400)
    params = O.init_params(cfg)
    rng = np.random.default_rng(5)
    params = [p if p.ndim == 2 else (0.01 * rng.standard_normal(p.shape)).astype(np.float32) for p in params]
    eps = rng.standard_normal((1, B, cfg.Z)).astype(np.float32)
    ctx = _lib.Context(784, 500, 20, B, B_global=Bg, row_offset=off, keep_grads=True, max_eval_rows=100)
    if with_comm:
        ctx.comm_init(_lib.Context.comm_unique_id(), 0, 1)
        assert ctx.comm_count() == 1
    ctx.set_data(x)
    ctx.set_params(O.flatten(params))
    ctx.set_eps_mode(_lib.EPS_HOST)
    ctx.push_eps(eps)
    b = 2
    elbo = ctx.update(b)
    rows = x[b * Bg + off:b * Bg + off + B].astype(np.float64)
    p64 = [p.astype(np.float64) for p in params]
    ref_e, ref_p, _, aux = O.step(p64, [np.zeros_like(p) for p in p64], rows, eps.astype(np.float64), cfg)
    assert abs(elbo * Bg - ref_e * B) <= 1e-4 * abs(ref_e * B), (elbo * Bg, ref_e * B)
    g = ctx.get_grads()
    for (n, s), gg, rr in zip(O.param_shapes(cfg), O.unflatten(g, cfg), aux["data_grads"]):
        assert rel(gg.reshape(s), rr) <= 1e-4, n
    check_theta(ctx.get_params(), O.flatten(ref_p), cfg.lr)
    ctx.close()


@pytest.mark.parametrize("n", [1, 2, 3, 20, 37, 69])
def test_graph_replay_any_length_equals_eager(n):
    """Replays of the captured step family (uploaded at capture) equal eager launches bitwise,
    for any call length."""
    from vaeb_amd import _lib
    cfg = O.Config(D=784, H=500, Z=20)
    x = O.synthetic_mnist(n=2000)
    order = np.random.default_rng(n).integers(0, 20, n).astype(np.int32)
    outs = []
    for use_graph in (True, False):
        ctx = _lib.Context(784, 500, 20, 100, use_graph=use_graph, max_eval_rows=100)
        ctx.set_data(x)
        ctx.set_params(O.flatten(O.init_params(cfg)))
        ctx.set_eps_mode(_lib.EPS_PHILOX, 10)
        ctx.set_step(0)
        ctx.update_many(order[:1])          # leave the context on arena 1 before the call
        ctx.update_many(order)
        outs.append((ctx.epoch_elbo(), ctx.get_params(), ctx.get_step()))
        ctx.close()
    assert outs[0][0] == outs[1][0]
    assert np.array_equal(outs[0][1], outs[1][1])
    assert outs[0][2] == outs[1][2] == n + 1


def test_host_eps_mode_rejects_multi_step_calls():
    from vaeb_amd import _lib
    ctx = _lib.Context(37, 19, 3, 13, max_eval_rows=13)
    ctx.set_data(O.synthetic_mnist(n=52, D=37))
    ctx.set_eps_mode(_lib.EPS_HOST)
    ctx.push_eps(np.zeros((1, 13, 3), np.float32))
    with pytest.raises(_lib.VaebError, match="one step per call"):
        ctx.update_many(np.array([0, 1], np.int32))
    ctx.update_many(np.array([0], np.int32))
    ctx.close()


def test_fullbayes_vae_matches_oracle_mnist20():
    """VAEBfullbayes.VAE at config 4's MNIST 784-500-20: theta0 is the single-draw init,
    3 steps (one eps draw each, from the host RandomStreams emulation) and validate match
    the oracle's mean_map objective: ELBO 1e-4 relative, theta' to 1e-3 lr."""
    from vaeb_amd.fullbayes import VAE
    from vaeb_amd.model import TheanoStreamEmulation
    cfg = O.Config(D=784, H=500, Z=20, objective="mean_map")
    x = O.synthetic_mnist(n=500)
    xv = O.synthetic_mnist(n=300, seed=4)
    m = VAE(x, False, 500, 20, rng="theano", max_eval_rows=100)
    theta0 = O.init_params_fullbayes(cfg)
    assert all(np.array_equal(p.get_value(), t) for p, t in zip(m.params, theta0))
    assert [p.name for p in m.params] == cfg.names
    stream = TheanoStreamEmulation(1, 10)
    p64 = [t.astype(np.float64) for t in theta0]
    a64 = [np.zeros_like(t) for t in p64]
    for b in (3, 0, 4):
        eps = stream.draw(100, 20)
        got = m.update(b)
        ref, p64, a64, _ = O.step(p64, a64, x[b * 100:(b + 1) * 100].astype(np.float64), eps.astype(np.float64), cfg)
        assert abs(got - ref) <= 1e-4 * abs(ref), (got, ref)
    check_theta(np.concatenate([p.get_value().ravel() for p in m.params]), O.flatten(p64), cfg.lr, frac=1e-3)
    epsv = stream.draw(300, 20)
    v = m.validate(xv)
    ref_v = O.validate(p64, xv.astype(np.float64), epsv.astype(np.float64), cfg)   # the mean
    assert abs(v - ref_v) <= 1e-4 * abs(ref_v), (v, ref_v)
    assert len(m.ADA) == len(m.params)
    m.close()


def test_native_checkpoint_resume_is_bit_identical(tmp_path):
    from vaeb_amd import _lib
    cfg = O.Config(D=560, H=200, Z=2, continuous=True)
    x = O.synthetic_frey(n=1500)
    order = np.random.default_rng(8).integers(0, 15, 61).astype(np.int32)
    theta0 = O.flatten(O.init_params(cfg))

    def fresh(seed=10, objective=_lib.OBJ_SUM_PRIOR):
        c = _lib.Context(560, 200, 2, 100, decoder=_lib.DEC_GAUSSIAN, max_eval_rows=100, objective=objective)
        c.set_data(x)
        c.set_params(theta0)
        c.set_eps_mode(_lib.EPS_PHILOX, seed)
        c.set_step(0)
        return c

    a = fresh()
    a.update_many(order[:29])            # odd: the writer sits on parameter arena 1
    f = str(tmp_path / "run.ckpt")
    # a NULL path is only a non-writing rank's part of a multi-rank gather
    with pytest.raises(_lib.VaebError, match="null path"):
        a.checkpoint_save(None)
    a.checkpoint_save(f)
    a.epoch_elbo()
    a.update_many(order[29:])
    ea = a.epoch_elbo()
    pa, acc_a, sa = a.get_params(), a.get_adagrad_state(), a.get_step()
    a.close()
    # another seed, with its steps already captured as graphs: the load must overwrite
    # everything, the captured seed included
    b = fresh(seed=77)
    b.update_many(order[:3])
    b.checkpoint_load(f)
    assert b.get_step() == 29
    b.epoch_elbo()
    b.update_many(order[29:])
    assert b.epoch_elbo() == ea
    assert np.array_equal(b.get_params(), pa) and np.array_equal(b.get_adagrad_state(), acc_a)
    assert b.get_step() == sa
    b.close()
    # a checkpoint of another shape is refused
    c = _lib.Context(784, 500, 20, 100, max_eval_rows=100)
    with pytest.raises(_lib.VaebError, match="checkpoint"):
        c.checkpoint_load(f)
    c.close()
    # ... and so is one written under another objective
    d = fresh(objective=_lib.OBJ_MEAN_MAP)
    with pytest.raises(_lib.VaebError, match="objective"):
        d.checkpoint_load(f)
    d.close()


@pytest.mark.parametrize("eps_mode", ["host", "philox"])
def test_resident_validation_equals_host_validate(eps_mode):
    from vaeb_amd import _lib
    cfg = O.Config(D=784, H=500, Z=20)
    xv = O.synthetic_mnist(n=2500, seed=6)
    params = O.init_params(cfg)
    ctx = _lib.Context(784, 500, 20, 100, max_eval_rows=1000)   # 3 device chunks
    ctx.set_data(O.synthetic_mnist(n=500))
    ctx.set_params(O.flatten(params))
    ctx.set_valid_data(xv)
    if eps_mode == "host":
        eps = np.random.default_rng(3).standard_normal((1, 2500, 20)).astype(np.float32)
        ctx.set_eps_mode(_lib.EPS_HOST)
        ctx.push_eps(eps)
    else:
        ctx.set_eps_mode(_lib.EPS_PHILOX, 10)
    v_host = ctx.validate(xv)
    v_res = ctx.validate_resident()
    assert v_res == v_host
    if eps_mode == "host":
        ref = O.validate([q.astype(np.float64) for q in params], xv.astype(np.float64), eps.astype(np.float64), cfg)
        assert abs(v_res - ref) <= 1e-4 * abs(ref)
    ctx.comm_init(_lib.Context.comm_unique_id(), 0, 1)   # world-1 all-reduce of the scalar
    assert ctx.validate_resident() == v_res
    ctx.close()


def test_fv_literal_step_mnist20():
    """Literal --full_varational at config 4's MNIST 784-500-20 against oracle.fv_step."""
    from vaeb_amd import _lib
    cfg = O.Config(D=784, H=500, Z=20, estimator="FV")
    B = 100
    x = O.synthetic_mnist(n=1000)
    rng = np.random.default_rng(14)
    theta = [(t + 0.02 * rng.standard_normal(t.shape)).astype(np.float32) for t in O.init_params(cfg)]
    flat = O.flatten(theta)
    ctx = _lib.Context(784, 500, 20, B, estimator=_lib.EST_FV, max_eval_rows=200)
    ctx.set_data(x)
    ctx.set_params(flat)
    ctx.set_fv_state(flat, np.full_like(flat, 1e-3), np.zeros_like(flat), np.zeros_like(flat))
    ctx.set_eps_mode(_lib.EPS_HOST)
    t64 = [q.astype(np.float64) for q in theta]
    m64 = [q.copy() for q in t64]
    s64 = [np.full_like(q, 1e-3) for q in t64]
    am64 = [np.zeros_like(q) for q in t64]
    as64 = [np.zeros_like(q) for q in t64]
    for t in range(3):
        eps = rng.standard_normal((1, B, 20)).astype(np.float32)
        ctx.push_eps(eps)
        e = ctx.update(t + 2)
        ref, m64, s64, am64, as64, _ = O.fv_step(t64, m64, s64, am64, as64, x[(t + 2) * B:(t + 3) * B].astype(np.float64),
                                                 eps.astype(np.float64), cfg)
        assert abs(e - ref) <= 1e-4 * abs(ref), (t, e, ref)
    gm, gs, _, _ = ctx.get_fv_state()
    assert np.abs(gm - O.flatten(m64)).max() <= 1e-6
    assert np.abs(gs - O.flatten(s64)).max() <= 1e-7
    assert np.array_equal(ctx.get_params(), flat)
    ctx.close()


@pytest.mark.parametrize("engine", ["f32", "bf16"])
@pytest.mark.parametrize("scaling", ["weak", "strong"])
def test_two_rank_decomposition_on_the_hip_path(scaling, engine):
    """The data-parallel decomposition with the real kernels, on one GPU: two contexts play
    ranks 0 and 1 of a world of 2 (the RCCL all-reduce itself needs one GPU per rank).  The
    SUM of their data gradients and SGVB values equals one context's on the whole global
    minibatch (VAEB.py:340-344: the objective is a sum over rows); Philox noise is keyed by
    the global row, so the ranks draw the single context's eps.  fp32 engine at MNIST
    784-500-20 (1e-5: only the accumulation order differs); bf16 engine at 256-128-32 (1e-3:
    its split-K slab counts depend on the rows per rank, so a few bf16 roundings differ)."""
    from vaeb_amd import _lib
    from vaeb_amd.dp import row_split
    bf = engine == "bf16"
    cfg = O.Config(D=256, H=128, Z=32) if bf else O.Config(D=784, H=500, Z=20)
    Bg = (256 if bf else 100) * (2 if scaling == "weak" else 1)
    x = O.synthetic_mnist(n=4 * Bg, D=cfg.D)
    theta = O.flatten(O.init_params(cfg))
    tol = 1e-3 if bf else 1e-5

    def run(B, off, B_global):
        c = _lib.Context(cfg.D, cfg.H, cfg.Z, B, B_global=B_global, row_offset=off, keep_grads=True,
                         max_eval_rows=B, dtype=_lib.DTYPE_BF16 if bf else _lib.DTYPE_F32)
        c.comm_init(_lib.Context.comm_unique_id(), 0, 1)   # the DP path: gradients stored, then reduced
        c.set_data(x)
        c.set_params(theta)
        c.set_eps_mode(_lib.EPS_PHILOX, 10)
        c.set_step(3)
        e = c.update(2)
        g = c.get_grads()
        c.close()
        return e, g

    full_e, full_g = run(Bg, 0, Bg)
    parts = [run(*row_split(Bg if scaling == "strong" else Bg // 2, 2, r, scaling)) for r in range(2)]
    # each rank reports its local SGVB / B_global
    assert abs(sum(p[0] for p in parts) - full_e) <= tol * abs(full_e)
    gsum = parts[0][1] + parts[1][1]
    for (n, s), a, b in zip(O.param_shapes(cfg), O.unflatten(gsum, cfg), O.unflatten(full_g, cfg)):
        assert rel(a, b) <= tol, (n, rel(a, b))
