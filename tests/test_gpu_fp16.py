"""Parity of the fp16 instantiation of the 16-bit engine (dtype=VAEB_DTYPE_F16: fp16 operands on
v_mfma_f32_16x16x32_f16, fp32 accumulation, fp32 master weights and Adagrad state; BASELINE
config 5 names "fp16 MFMA") against the CPU oracle, through the C ABI.  The same kernels as the
bf16 engine (h16_engines.hpp instantiates gemm_bf16.hpp / step_bf16.hpp / thin_bf16.hpp twice);
what differs is the 16-bit format and, for the mean objective, the backward's loss scale.

References and tolerances (the bf16 module's, tightened where fp16's 11-bit significand allows):
  * the oracle with q = fp16_round at exactly the engine's 16-bit storage points, float64:
      ELBO relative <= 1e-4, data gradients norm-wise relative <= 2e-3 per tensor,
      Adagrad accumulator relative <= 4e-3;
  * the plain float64 oracle: ELBO relative <= 2e-3, gradients norm-wise <= 2e-2 (bf16: 1e-2 / 8e-2);
  * the mean objective (VAEBfullbayes.py:142) divides every data gradient by B_global: at
    B = 8192 the backward's dA1 falls below fp16's smallest normal (6.1e-5), so the engine
    carries its 16-bit backward operands scaled by S = 2^13 (engine_bf16.inc h16_scale) and
    unscales in fp32; its oracle is q = fp16_round_scaled(S).
GEMMs alone: |C - ref| <= 1e-5 (|A| |B|) elementwise against float64 products of fp16-rounded
operands, every layout, tails, split-K and the 8-phase loop.
"""
import numpy as np
import pytest

from oracle import vaeb_oracle as O

pytestmark = pytest.mark.gpu

EST = {"LB": 0, "LA": 1}
OBJ = {"sum_prior": 0, "mean_map": 1}


def rel(a, b):
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


@pytest.fixture(scope="module")
def hctx():
    from vaeb_amd import _lib
    c = _lib.Context(64, 32, 8, 16, dtype=_lib.DTYPE_F16)
    yield c
    c.close()


@pytest.mark.parametrize("ako,bko", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("M,N,K,ks", [(256, 128, 512, 1), (200, 136, 328, 3), (296, 520, 328, -1), (512, 512, 4096, -2),
                                      (8, 520, 4096, 4)])
def test_fp16_gemm_layouts(hctx, ako, bko, M, N, K, ks):
    rng = np.random.default_rng(M + 7 * N + K + 10 * ako + 20 * bko)
    A = rng.standard_normal((M, K)).astype(np.float32)
    B = rng.standard_normal((K, N)).astype(np.float32)
    As = A.T.copy() if ako else A
    Bs = B if bko else B.T.copy()
    C = hctx.test_gemm_bf16(As, Bs, ako, bko, M, N, K, ks)
    Aq = O.fp16_round(A).astype(np.float64)
    Bq = O.fp16_round(B).astype(np.float64)
    ref = Aq @ Bq
    bound = 1e-5 * (np.abs(Aq) @ np.abs(Bq)) + 1e-30
    assert np.all(np.abs(C - ref) <= bound), float(np.max(np.abs(C - ref) / bound))
    # the operands really are fp16 (11-bit significand), not bf16: a bf16-rounded product is
    # further from the engine's than the fp16 bound allows
    Ab = O.bf16_round(A).astype(np.float64)
    Bb = O.bf16_round(B).astype(np.float64)
    assert np.max(np.abs(C - Ab @ Bb) / bound) > 1.0


CASES = [
    ("bern_LB", dict(D=512, H=256, Z=32), 512),
    ("gauss_LA_L2", dict(D=256, H=256, Z=16, continuous=True, estimator="LA", L=2), 512),
    ("bern_LB_tails", dict(D=520, H=264, Z=24), 1100),
    ("bern_mean_map", dict(D=512, H=256, Z=32, objective="mean_map"), 1024),
]


def make_ctx(cfg, B, keep_grads=True):
    from vaeb_amd import _lib
    return _lib.Context(cfg.D, cfg.H, cfg.Z, B, L=cfg.L, decoder=int(cfg.continuous), estimator=EST[cfg.estimator],
                        objective=OBJ[cfg.objective], lr=cfg.lr, keep_grads=keep_grads, max_eval_rows=512,
                        dtype=_lib.DTYPE_F16)


def data_for(cfg, n, seed=0):
    if cfg.continuous:
        return O.synthetic_frey(n=n, D=cfg.D, seed=seed)
    return O.synthetic_mnist(n=n, D=cfg.D, seed=seed)


def loss_scale(cfg, B):
    """engine_bf16.inc h16_scale: the largest power of two <= B_global for the mean objective."""
    return float(2 ** int(np.floor(np.log2(B)))) if cfg.objective == "mean_map" else 1.0


def one_step(cfg, B, x, params, acc, eps, idx=1):
    ctx = make_ctx(cfg, B)
    ctx.set_data(x)
    ctx.set_params(O.flatten(params))
    ctx.set_adagrad_state(O.flatten(acc))
    ctx.set_eps_mode(1)
    ctx.push_eps(eps)
    elbo = ctx.update(idx)
    out = (elbo, ctx.get_grads(), ctx.get_adagrad_state(), ctx.get_params())
    ctx.close()
    return out


def check_theta(cfg, params, acc, g, newp):
    """theta' is the fp32 Adagrad rule applied to the engine's own (unscaled) gradient."""
    th = O.flatten(params).astype(np.float64)
    prior = 1.0 if cfg.objective == "sum_prior" else 0.0
    gt = g.astype(np.float64) - prior * th
    want = th + cfg.lr * gt / (np.sqrt(O.flatten(acc).astype(np.float64) + gt * gt) + cfg.eps)
    if cfg.objective == "mean_map":
        want = want - cfg.lr * cfg.eps * th * th
    assert np.abs(newp - want).max() <= 1e-6 + 1e-5 * np.abs(want).max()


@pytest.mark.parametrize("name,kw,B", CASES, ids=[c[0] for c in CASES])
def test_fp16_step_parity(name, kw, B):
    cfg = O.Config(**kw)
    x = data_for(cfg, 3 * B)
    rng = np.random.default_rng(5)
    params = [p if p.ndim == 2 else (0.01 * rng.standard_normal(p.shape)).astype(np.float32)
              for p in O.init_params(cfg)]
    acc = [np.full_like(p, 1e-3) for p in params]
    eps = rng.standard_normal((cfg.L, B, cfg.Z)).astype(np.float32)
    elbo, g, newa, newp = one_step(cfg, B, x, params, acc, eps)
    p64 = [p.astype(np.float64) for p in params]
    a64 = [a.astype(np.float64) for a in acc]
    xb = x[B:2 * B].astype(np.float64)
    q = O.fp16_round_scaled(loss_scale(cfg, B)) if cfg.objective == "mean_map" else O.fp16_round
    q_elbo, _, q_a, q_aux = O.step(p64, a64, xb, eps.astype(np.float64), cfg, q=q)
    f_elbo, _, _, f_aux = O.step(p64, a64, xb, eps.astype(np.float64), cfg)
    assert abs(elbo - q_elbo) <= 1e-4 * abs(q_elbo), (elbo, q_elbo)
    assert abs(elbo - f_elbo) <= 2e-3 * abs(f_elbo), (elbo, f_elbo)
    for (n, s), gg, rq, rf in zip(O.param_shapes(cfg), O.unflatten(g, cfg), q_aux["data_grads"], f_aux["data_grads"]):
        assert rel(gg.reshape(s), rq) <= 2e-3, (n, rel(gg.reshape(s), rq))
        assert rel(gg.reshape(s), rf) <= 2e-2, (n, rel(gg.reshape(s), rf))
    assert rel(newa, O.flatten(q_a)) <= 4e-3
    check_theta(cfg, params, acc, g, newp)


def test_fp16_mean_objective_loss_scale_keeps_small_gradients():
    """The mean objective at B = 8192 (config 5's batch): the oracle's dA1 is below fp16's
    smallest normal for most elements, so an unscaled fp16 backward would keep a few mantissa
    bits of them at best.  The engine (S = 2^13) matches the float64 oracle as closely as the
    sum objective does (gradients norm-wise <= 2e-2, dW1 / dW3 -- the ones fed by dA1 / dA3 --
    included), and the unscaled-fp16 oracle is measurably worse on them."""
    cfg = O.Config(D=512, H=256, Z=32, objective="mean_map")
    B = 8192
    x = data_for(cfg, 2 * B)
    rng = np.random.default_rng(9)
    params = [p if p.ndim == 2 else (0.01 * rng.standard_normal(p.shape)).astype(np.float32)
              for p in O.init_params(cfg)]
    acc = [np.full_like(p, 1e-3) for p in params]
    eps = rng.standard_normal((1, B, cfg.Z)).astype(np.float32)
    elbo, g, newa, newp = one_step(cfg, B, x, params, acc, eps)
    p64 = [p.astype(np.float64) for p in params]
    a64 = [a.astype(np.float64) for a in acc]
    xb = x[B:].astype(np.float64)
    out = O.forward_backward(p64, xb, eps.astype(np.float64), cfg)
    assert np.median(np.abs(out["dA1"])) < 6.1e-5, np.median(np.abs(out["dA1"]))
    f_elbo, _, _, f_aux = O.step(p64, a64, xb, eps.astype(np.float64), cfg)
    _, _, _, u_aux = O.step(p64, a64, xb, eps.astype(np.float64), cfg, q=O.fp16_round)   # no loss scale
    assert abs(elbo - f_elbo) <= 2e-3 * abs(f_elbo), (elbo, f_elbo)
    errs = {}
    for (n, s), gg, rf, ru in zip(O.param_shapes(cfg), O.unflatten(g, cfg), f_aux["data_grads"], u_aux["data_grads"]):
        errs[n] = (rel(gg.reshape(s), rf), rel(ru, rf))
        assert errs[n][0] <= 2e-2, (n, errs[n])
    assert errs["W1"][0] < errs["W1"][1] and errs["W3"][0] < errs["W3"][1], errs
    check_theta(cfg, params, acc, g, newp)


def test_fp16_graph_epoch_matches_eager_and_tracks_f32():
    """10 steps with device Philox noise: graph replay == eager launches bit for bit; the epoch
    ELBO tracks the fp32 engine on the same noise within 5e-3."""
    from vaeb_amd import _lib
    cfg = O.Config(D=256, H=128, Z=32)
    B = 256
    x = data_for(cfg, 8 * B)
    params = O.flatten(O.init_params(cfg))
    order = np.array([3, 1, 4, 1, 5, 7, 2, 6, 0, 2], np.int32)
    res = {}
    for mode, kw in (("graph", dict(use_graph=True, dtype=_lib.DTYPE_F16)),
                     ("eager", dict(use_graph=False, dtype=_lib.DTYPE_F16)),
                     ("f32", dict(use_graph=True, dtype=_lib.DTYPE_F32))):
        ctx = _lib.Context(cfg.D, cfg.H, cfg.Z, B, max_eval_rows=B, **kw)
        ctx.set_data(x)
        ctx.set_params(params)
        ctx.set_eps_mode(0, seed=10)
        ctx.update_many(order)
        s, n = ctx.epoch_elbo()
        res[mode] = (s / n, ctx.get_params())
        ctx.close()
    assert res["graph"][0] == res["eager"][0]
    assert np.array_equal(res["graph"][1], res["eager"][1])
    assert abs(res["graph"][0] - res["f32"][0]) <= 5e-3 * abs(res["f32"][0])


@pytest.mark.parametrize("dt", ["fp16", "bf16"])
def test_binary_dataset_bit_tile_is_bitwise_the_16bit_tile(dt):
    """A binary dataset (every value 0 or 1, D % 32 == 0) is also kept as bits, and the Bernoulli
    decoder epilogue expands its x tile from them (gemm_bf16.hpp EpiDecOutT::load_in).  The same
    rows with one extra, never-sampled row of 0.5 appended take the 16-bit x tile instead.  Graph
    and eager steps on either must agree bit for bit -- theta, Adagrad state, epoch ELBO --
    including a tail tile past D (D = 544: 17 words, the tile's last 7 read nothing) and rows past
    the batch (B = 100)."""
    from vaeb_amd import _lib
    cfg = O.Config(D=544, H=264, Z=40)
    B = 100
    x = data_for(cfg, 8 * B)
    assert set(np.unique(x)) <= {0.0, 1.0}
    xg = np.concatenate([x, np.full((1, cfg.D), 0.5, np.float32)])   # not binary: the 16-bit tile
    params = O.flatten(O.init_params(cfg))
    order = np.array([3, 1, 4, 1, 5, 7, 2, 6, 0, 2], np.int32)
    res = {}
    for data_name, data in (("bits", x), ("half", xg)):
        for use_graph in (True, False):
            ctx = _lib.Context(cfg.D, cfg.H, cfg.Z, B, max_eval_rows=B, use_graph=use_graph,
                               dtype=_lib.DTYPE_F16 if dt == "fp16" else _lib.DTYPE_BF16)
            ctx.set_data(data)
            ctx.set_params(params)
            ctx.set_eps_mode(0, seed=10)
            ctx.update_many(order)
            s, n = ctx.epoch_elbo()
            res[data_name, use_graph] = (s / n, ctx.get_params(), ctx.get_adagrad_state())
            ctx.close()
    ref = res["half", True]
    for key, got in res.items():
        assert got[0] == ref[0], key
        assert np.array_equal(got[1], ref[1]), key
        assert np.array_equal(got[2], ref[2]), key


def test_fp16_validate_and_reconstruct():
    cfg = O.Config(D=256, H=128, Z=32)
    B = 128
    x = data_for(cfg, 4 * B)
    params = O.init_params(cfg)
    ctx = make_ctx(cfg, B, keep_grads=False)
    ctx.set_data(x)
    ctx.set_params(O.flatten(params))
    ctx.set_eps_mode(1)
    xv = x[:300]
    eps = np.random.default_rng(1).standard_normal((1, 300, cfg.Z)).astype(np.float32)
    ctx.push_eps(eps)
    got = ctx.validate(xv)
    p64 = [p.astype(np.float64) for p in params]
    ref = O.validate(p64, xv.astype(np.float64), eps.astype(np.float64), cfg, q=O.fp16_round)
    assert abs(got - ref) <= 1e-4 * abs(ref), (got, ref)
    y = ctx.reconstruct(xv)
    out = O.forward_backward(p64, xv.astype(np.float64), np.zeros((1, 300, cfg.Z)), cfg, need_grad=False,
                             q=O.fp16_round)
    assert np.abs(y - out["y"]).max() <= 5e-4
    ctx.close()


def test_fp16_full_size_step_matches_rounded_oracle():
    """Config 5 at the size BASELINE names (4096-2048-128, B = 8192, x ~ Bernoulli(0.5)) with fp16
    operands, one step against the float64 oracle with fp16 rounding at the engine's rounding
    points: ELBO 1e-4, data gradients 2e-3 per tensor, Adagrad accumulator 4e-3; theta' is the
    fp32 Adagrad rule on the engine's own gradient."""
    from vaeb_amd import _lib
    D, H, Z, B = 4096, 2048, 128, 8192
    cfg = O.Config(D=D, H=H, Z=Z)
    rng = np.random.default_rng(11)
    x = (rng.random((2 * B, D), dtype=np.float32) < 0.5).astype(np.float32)
    params = [p if p.ndim == 2 else (0.01 * rng.standard_normal(p.shape)).astype(np.float32)
              for p in O.init_params(cfg)]
    acc = [np.full_like(p, 1e-3) for p in params]
    eps = rng.standard_normal((1, B, Z)).astype(np.float32)
    ctx = _lib.Context(D, H, Z, B, keep_grads=True, max_eval_rows=B, dtype=_lib.DTYPE_F16)
    ctx.set_data(x)
    ctx.set_params(O.flatten(params))
    ctx.set_adagrad_state(O.flatten(acc))
    ctx.set_eps_mode(_lib.EPS_HOST)
    ctx.push_eps(eps)
    elbo = ctx.update(1)
    g, newa, newp = ctx.get_grads(), ctx.get_adagrad_state(), ctx.get_params()
    ctx.close()
    p64 = [p.astype(np.float64) for p in params]
    q_elbo, _, q_a, q_aux = O.step(p64, [a.astype(np.float64) for a in acc], x[B:].astype(np.float64),
                                   eps.astype(np.float64), cfg, q=O.fp16_round)
    assert abs(elbo - q_elbo) <= 1e-4 * abs(q_elbo), (elbo, q_elbo)
    for (n, s), gg, rq in zip(O.param_shapes(cfg), O.unflatten(g, cfg), q_aux["data_grads"]):
        assert rel(gg.reshape(s), rq) <= 2e-3, (n, rel(gg.reshape(s), rq))
    assert rel(newa, O.flatten(q_a)) <= 4e-3
    check_theta(cfg, params, acc, g, newp)


@pytest.mark.parametrize("overlap,fork,shard", [("1", "1", "1"), ("0", "0", "0")])
def test_fp16_dp_path_world1_matches_fused_optimizer(overlap, fork, shard, monkeypatch):
    """The data-parallel path (gradients stored unscaled, RCCL all-reduce, Adagrad + fp16 shadow
    in adagrad_bf16_kernel) at world size 1 against the fused-optimizer path, 6 steps."""
    from vaeb_amd import _lib
    monkeypatch.setenv("VAEB_DP_OVERLAP", overlap)
    monkeypatch.setenv("VAEB_BF_FORK", fork)
    monkeypatch.setenv("VAEB_DP_SHARD", shard)
    cfg = O.Config(D=256, H=128, Z=32)
    B = 256
    x = data_for(cfg, 8 * B)
    order = np.array([3, 1, 4, 1, 5, 7], np.int32)
    outs = []
    for use_comm in (False, True):
        ctx = _lib.Context(cfg.D, cfg.H, cfg.Z, B, max_eval_rows=B, dtype=_lib.DTYPE_F16)
        if use_comm:
            ctx.comm_init(_lib.Context.comm_unique_id(), 0, 1)
        ctx.set_data(x)
        ctx.set_params(O.flatten(O.init_params(cfg)))
        ctx.set_eps_mode(_lib.EPS_PHILOX, 10)
        ctx.set_step(0)
        ctx.update_many(order)
        s, n = ctx.epoch_elbo()
        outs.append((s / n, ctx.get_params(), ctx.get_adagrad_state()))
        ctx.close()
    assert abs(outs[0][0] - outs[1][0]) <= 1e-5 * abs(outs[0][0]), (outs[0][0], outs[1][0])
    assert np.abs(outs[0][1] - outs[1][1]).max() <= 1e-5
    assert rel(outs[1][2], outs[0][2]) <= 1e-4
