"""Parity of the bf16 large-batch engine (dtype=VAEB_DTYPE_BF16, vaeb_amd/csrc/gemm_bf16.hpp,
step_bf16.hpp; BASELINE config 5) against the CPU oracle, through the C ABI.

Two references:
  * the oracle with `q=bf16_round` -- the same algorithm with bf16 storage rounding at
    exactly the engine's rounding points, evaluated in float64.  Tolerances (fp32
    accumulation order and the ~1-ulp hardware transcendentals remain; a value within
    ~1e-7 of a bf16 rounding tie can round the other way):
      ELBO relative <= 1e-4, data gradients norm-wise relative <= 2e-3 per tensor,
      Adagrad accumulator relative <= 4e-3;
  * the plain float64 oracle (no rounding) -- bounds the bf16 error itself:
      ELBO relative <= 1e-2, gradients norm-wise relative <= 8e-2.
The GEMM engine alone is checked against float64 products of bf16-rounded operands at
|C - ref| <= 1e-5 * (|A| |B|) elementwise, for all four operand layouts, tails and
split-K.
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
def gctx():
    from vaeb_amd import _lib
    c = _lib.Context(64, 32, 8, 16, dtype=_lib.DTYPE_BF16)
    yield c
    c.close()


GEMM_SHAPES = [(256, 128, 512, 1), (200, 136, 328, 1), (200, 136, 328, 3), (64, 40, 72, 2), (8, 520, 4096, 4)]


@pytest.mark.parametrize("ako,bko", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("M,N,K,ks", GEMM_SHAPES)
def test_gemm_layouts(gctx, ako, bko, M, N, K, ks):
    rng = np.random.default_rng(M + 7 * N + K + ks + 10 * ako + 20 * bko)
    A = rng.standard_normal((M, K)).astype(np.float32)   # logical [M, K]
    B = rng.standard_normal((K, N)).astype(np.float32)   # logical [K, N]
    As = A.T.copy() if ako else A                         # stored layout
    Bs = B if bko else B.T.copy()
    C = gctx.test_gemm_bf16(As, Bs, ako, bko, M, N, K, ks)
    Aq = O.bf16_round(A).astype(np.float64)
    Bq = O.bf16_round(B).astype(np.float64)
    ref = Aq @ Bq
    bound = 1e-5 * (np.abs(Aq) @ np.abs(Bq)) + 1e-30
    assert np.all(np.abs(C - ref) <= bound), float(np.max(np.abs(C - ref) / bound))


GEMM8_SHAPES = [(256, 256, 512, 1), (296, 520, 328, 1), (512, 512, 4096, 2), (200, 136, 64, 1), (8, 520, 4096, 4),
                (768, 256, 1000, 3)]


@pytest.mark.parametrize("ako,bko", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("M,N,K,ks", GEMM8_SHAPES)
def test_gemm8_layouts(gctx, ako, bko, M, N, K, ks):
    """The 256 x 256 8-phase main loop (gemm8_kernel: BK = 64, two K-tile buffers, one
    half-tile staged per phase, staggered wave groups) on every operand layout, partial
    tiles, K tails (K % 64 != 0), one-K-tile slices and split-K, same bound as above."""
    rng = np.random.default_rng(3 * M + 5 * N + K + ks + 10 * ako + 20 * bko)
    A = rng.standard_normal((M, K)).astype(np.float32)
    B = rng.standard_normal((K, N)).astype(np.float32)
    As = A.T.copy() if ako else A
    Bs = B if bko else B.T.copy()
    C = gctx.test_gemm_bf16(As, Bs, ako, bko, M, N, K, -ks)
    Aq = O.bf16_round(A).astype(np.float64)
    Bq = O.bf16_round(B).astype(np.float64)
    ref = Aq @ Bq
    bound = 1e-5 * (np.abs(Aq) @ np.abs(Bq)) + 1e-30
    assert np.all(np.abs(C - ref) <= bound), float(np.max(np.abs(C - ref) / bound))


CASES = [
    ("bern_LB", dict(D=256, H=128, Z=32), 256),
    ("bern_LB_tails", dict(D=200, H=136, Z=24), 200),
    ("gauss_LB", dict(D=256, H=96, Z=16, continuous=True), 192),
    ("bern_LA_L2", dict(D=128, H=64, Z=16, estimator="LA", L=2), 136),
    ("gauss_mean_map", dict(D=128, H=64, Z=8, continuous=True, objective="mean_map"), 128),
    ("synth_shape_small_batch", dict(D=4096, H=2048, Z=128), 128),
    # Z % 128 == 0, LB, L = 1: heads and dz run on the thin kernels with the latent block
    # fused (thin_bf16.hpp); row tails of the 64- / 32-row blocks, a K tail (H % 32 != 0)
    ("thin_tails", dict(D=264, H=200, Z=128), 200),
    ("thin_gauss_mean_map", dict(D=128, H=64, Z=256, continuous=True, objective="mean_map"), 96),
    # long-K weight gradients (K = L * B >= 1024) with row / column / K tails
    ("bern_LB_longk", dict(D=512, H=256, Z=32), 1024),
    ("gauss_LA_L2_longk", dict(D=256, H=256, Z=16, continuous=True, estimator="LA", L=2), 1024),
    ("bern_LB_longk_tails", dict(D=520, H=264, Z=24), 1100),
]


def make_ctx(cfg, B, keep_grads=True):
    from vaeb_amd import _lib
    return _lib.Context(cfg.D, cfg.H, cfg.Z, B, L=cfg.L, decoder=int(cfg.continuous), estimator=EST[cfg.estimator],
                        objective=OBJ[cfg.objective], lr=cfg.lr, keep_grads=keep_grads, max_eval_rows=512,
                        dtype=_lib.DTYPE_BF16)


def data_for(cfg, n, seed=0):
    if cfg.continuous:
        return O.synthetic_frey(n=n, D=cfg.D, seed=seed)
    return O.synthetic_mnist(n=n, D=cfg.D, seed=seed)


@pytest.mark.parametrize("name,kw,B", CASES, ids=[c[0] for c in CASES])
def test_bf16_step_parity(name, kw, B):
    cfg = O.Config(**kw)
    x = data_for(cfg, 3 * B)
    params = O.init_params(cfg)
    rng = np.random.default_rng(5)
    params = [p if p.ndim == 2 else (0.01 * rng.standard_normal(p.shape)).astype(np.float32) for p in params]
    acc = [np.full_like(p, 1e-3) for p in params]
    eps = rng.standard_normal((cfg.L, B, cfg.Z)).astype(np.float32)
    idx = 1
    xb = x[idx * B:(idx + 1) * B].astype(np.float64)

    ctx = make_ctx(cfg, B)
    ctx.set_data(x)
    ctx.set_params(O.flatten(params))
    ctx.set_adagrad_state(O.flatten(acc))
    ctx.set_eps_mode(1)
    ctx.push_eps(eps)
    elbo = ctx.update(idx)
    g = ctx.get_grads()
    newa = ctx.get_adagrad_state()
    newp = ctx.get_params()
    ctx.close()

    p64 = [p.astype(np.float64) for p in params]
    a64 = [a.astype(np.float64) for a in acc]
    e64 = eps.astype(np.float64)
    q_elbo, q_p, q_a, q_aux = O.step(p64, a64, xb, e64, cfg, q=O.bf16_round)
    f_elbo, _, _, f_aux = O.step(p64, a64, xb, e64, cfg)

    assert abs(elbo - q_elbo) <= 1e-4 * abs(q_elbo), (elbo, q_elbo)
    assert abs(elbo - f_elbo) <= 1e-2 * abs(f_elbo), (elbo, f_elbo)
    for (n, s), gg, rq, rf in zip(O.param_shapes(cfg), O.unflatten(g, cfg), q_aux["data_grads"], f_aux["data_grads"]):
        assert rel(gg.reshape(s), rq) <= 2e-3, (n, rel(gg.reshape(s), rq))
        assert rel(gg.reshape(s), rf) <= 8e-2, (n, rel(gg.reshape(s), rf))
    assert rel(newa, O.flatten(q_a)) <= 4e-3
    # the optimizer applied to the engine's own gradient reproduces theta' (fp32 rule)
    th = O.flatten(params).astype(np.float64)
    gg = g.astype(np.float64)
    prior = 1.0 if cfg.objective == "sum_prior" else 0.0
    gt = gg - prior * th
    a2 = O.flatten(acc).astype(np.float64) + gt * gt
    want = th + cfg.lr * gt / (np.sqrt(a2) + cfg.eps)
    if cfg.objective == "mean_map":
        want = want - cfg.lr * cfg.eps * th * th
    assert np.abs(newp - want).max() <= 1e-6 + 1e-5 * np.abs(want).max()


def test_bf16_validate_and_reconstruct():
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
    ref = O.validate(p64, xv.astype(np.float64), eps.astype(np.float64), cfg, q=O.bf16_round)
    assert abs(got - ref) <= 1e-4 * abs(ref), (got, ref)
    y = ctx.reconstruct(xv)
    out = O.forward_backward(p64, xv.astype(np.float64), np.zeros((1, 300, cfg.Z)), cfg, need_grad=False,
                             q=O.bf16_round)
    assert np.abs(y - out["y"]).max() <= 2e-3
    # posterior-sample reconstruction (VAEB.py:271-291), 2 samples over 3 device chunks
    eps2 = np.random.default_rng(2).standard_normal((2, 300, cfg.Z)).astype(np.float32)
    ctx.push_eps(eps2.reshape(1, 600, cfg.Z))
    ys = ctx.reconstruct_sampled(xv, 2)
    ref_s = O.reconstruct(p64, xv.astype(np.float64), eps2.astype(np.float64), cfg)
    assert np.abs(ys - ref_s).max() <= 2e-2
    ctx.close()


def test_bf16_graph_epoch_matches_eager_and_tracks_oracle():
    """10 steps with device Philox noise: graph replay == eager launches bit for bit; the
    epoch ELBO tracks the fp32 engine on the same noise within 1e-2."""
    from vaeb_amd import _lib
    cfg = O.Config(D=256, H=128, Z=32)
    B = 256
    x = data_for(cfg, 8 * B)
    params = O.flatten(O.init_params(cfg))
    order = np.array([3, 1, 4, 1, 5, 7, 2, 6, 0, 2], np.int32)
    res = {}
    for mode, kw in (("graph", dict(use_graph=True, dtype=_lib.DTYPE_BF16)),
                     ("eager", dict(use_graph=False, dtype=_lib.DTYPE_BF16)),
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
    assert abs(res["graph"][0] - res["f32"][0]) <= 1e-2 * abs(res["f32"][0])


def test_bf16_full_size_row_linearity_and_determinism():
    """Config 5 at its full size (4096-2048-128, B = 8192): size-independent properties,
    beside the oracle comparison at the same size (next test).  The SGVB and the data gradient
    are sums over rows (VAEB.py:340-344), so the full batch equals the sum of its two
    halves run as separate 4096-row steps (bf16 rounding is per element; only the fp32
    accumulation order differs: norm-wise <= 1e-3); and a repeated step is bit-identical."""
    from vaeb_amd import _lib
    D, H, Z, B = 4096, 2048, 128, 8192
    rng = np.random.default_rng(3)
    x = (rng.random((B, D), dtype=np.float32) < 0.5).astype(np.float32)
    cfg = O.Config(D=D, H=H, Z=Z)
    theta = O.flatten(O.init_params(cfg))
    eps = rng.standard_normal((1, B, Z)).astype(np.float32)

    def run(rows, e):
        ctx = _lib.Context(D, H, Z, rows.shape[0], keep_grads=True, max_eval_rows=rows.shape[0],
                           dtype=_lib.DTYPE_BF16)
        ctx.set_data(rows)
        ctx.set_params(theta)
        ctx.set_eps_mode(_lib.EPS_HOST)
        ctx.push_eps(e)
        elbo = ctx.update(0)
        out = (elbo * rows.shape[0], ctx.get_grads(), ctx.get_params())
        ctx.close()
        return out

    s_full, g_full, p_full = run(x, eps)
    s_a, g_a, _ = run(x[:B // 2], np.ascontiguousarray(eps[:, :B // 2]))
    s_b, g_b, _ = run(x[B // 2:], np.ascontiguousarray(eps[:, B // 2:]))
    assert np.all(np.isfinite(g_full))
    assert abs(s_full - (s_a + s_b)) <= 1e-4 * abs(s_full), (s_full, s_a + s_b)
    assert rel(g_full, g_a + g_b) <= 1e-3, rel(g_full, g_a + g_b)
    s_again, g_again, p_again = run(x, eps)
    assert s_again == s_full and np.array_equal(g_again, g_full) and np.array_equal(p_again, p_full)


def test_bf16_full_size_step_matches_rounded_oracle():
    """Config 5 at the size BASELINE names (4096-2048-128, B = 8192, x ~ Bernoulli(0.5) as
    bench.py's synth workload), one step against the float64 oracle with bf16 rounding at
    the engine's rounding points (O.step(..., q=bf16_round): ~7e11 FLOP, ~15 s on 8 host
    threads) at this module's tolerances: ELBO 1e-4, data gradients 2e-3 per tensor,
    Adagrad accumulator 4e-3; and theta' is the fp32 Adagrad rule applied to the engine's
    own gradient.  Complements the property test above."""
    from vaeb_amd import _lib
    D, H, Z, B = 4096, 2048, 128, 8192
    cfg = O.Config(D=D, H=H, Z=Z)
    rng = np.random.default_rng(11)
    x = (rng.random((2 * B, D), dtype=np.float32) < 0.5).astype(np.float32)
    params = O.init_params(cfg)
    params = [p if p.ndim == 2 else (0.01 * rng.standard_normal(p.shape)).astype(np.float32) for p in params]
    acc = [np.full_like(p, 1e-3) for p in params]
    eps = rng.standard_normal((1, B, Z)).astype(np.float32)
    ctx = _lib.Context(D, H, Z, B, keep_grads=True, max_eval_rows=B, dtype=_lib.DTYPE_BF16)
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
                                   eps.astype(np.float64), cfg, q=O.bf16_round)
    assert abs(elbo - q_elbo) <= 1e-4 * abs(q_elbo), (elbo, q_elbo)
    for (n, s), gg, rq in zip(O.param_shapes(cfg), O.unflatten(g, cfg), q_aux["data_grads"]):
        assert rel(gg.reshape(s), rq) <= 2e-3, (n, rel(gg.reshape(s), rq))
    assert rel(newa, O.flatten(q_a)) <= 4e-3
    th = O.flatten(params).astype(np.float64)
    gt = g.astype(np.float64) - th
    want = th + cfg.lr * gt / (np.sqrt(O.flatten(acc).astype(np.float64) + gt * gt) + cfg.eps)
    assert np.abs(newp - want).max() <= 1e-6 + 1e-5 * np.abs(want).max()


@pytest.mark.parametrize("overlap,fork,shard", [("1", "1", "0"), ("0", "1", "0"), ("1", "0", "0"),
                                                ("1", "1", "1"), ("0", "1", "1"), ("1", "0", "1")])
def test_bf16_dp_path_world1_matches_fused_optimizer(overlap, fork, shard, monkeypatch):
    """The data-parallel path of the bf16 engine (gradients stored, RCCL all-reduce of
    [grads | SGVB], replicated Adagrad + shadow rewrite in adagrad_bf16_kernel) at world
    size 1 against the fused-optimizer path, over 6 graph-replayed steps: forked (the
    default: dW1, dW2 | dW6, dW45 on the second stream, bucket A reduced and updated there
    right after dW2 -- or, without overlap, everything reduced after the join) and unforked."""
    from vaeb_amd import _lib
    monkeypatch.setenv("VAEB_DP_OVERLAP", overlap)
    monkeypatch.setenv("VAEB_BF_FORK", fork)
    monkeypatch.setenv("VAEB_DP_SHARD", shard)   # 1: the sharded optimizer forced at world 1
    cfg = O.Config(D=256, H=128, Z=32)
    B = 256
    x = data_for(cfg, 8 * B)
    order = np.array([3, 1, 4, 1, 5, 7], np.int32)
    outs = []
    for use_comm in (False, True):
        ctx = _lib.Context(cfg.D, cfg.H, cfg.Z, B, max_eval_rows=B, dtype=_lib.DTYPE_BF16)
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


@pytest.mark.parametrize("gauss", [False, True])
def test_bf16_forked_and_single_stream_steps_agree(monkeypatch, gauss):
    """the forked bf16 step (dW1, dW2 | dW6 and dW4 | dW5 on a second stream
    beside the dz -> [dMu | dLv] -> dh -> dW3 chain, joined by events inside the graph) and
    the single-stream step (VAEB_BF_FORK=0: dhd and dW2 in one grid) compute the same
    products with the same K order, so 10 Philox steps agree to 1e-6 in every parameter and
    the ELBO -- this pins the cross-stream ordering independently of the golden tolerances;
    graph replay and eager launches agree bitwise for each form.  Bernoulli and Gaussian (the
    [W2 | W6] interleave).  (The other fork points and the split dW2 of round 5 were removed in
    round 6 as measured slower.)"""
    # the forked dhd on the transposed product (VAEB_BF_DTT=1, the default) adds its bias column
    # sums in another order than the single-stream grid: compared with DTT=0 here, and DTT=1
    # against DTT=0 in test_bf16_tile_form_switches_agree
    monkeypatch.setenv("VAEB_BF_DTT", "0")
    from vaeb_amd import _lib
    cfg = O.Config(D=512, H=256, Z=32, continuous=gauss)
    B = 512
    x = (np.random.default_rng(4).random((6 * B, cfg.D)) < 0.4).astype(np.float32)
    order = np.array([3, 1, 4, 1, 5, 0, 2, 5, 3, 4], np.int32)
    out = {}
    for fork in ("1", "0"):
        for use_graph in (True, False):
            monkeypatch.setenv("VAEB_BF_FORK", fork)
            ctx = _lib.Context(cfg.D, cfg.H, cfg.Z, B, decoder=int(gauss), max_eval_rows=B, dtype=_lib.DTYPE_BF16,
                               use_graph=use_graph)
            ctx.set_data(x)
            ctx.set_params(O.flatten(O.init_params(cfg)))
            ctx.set_eps_mode(_lib.EPS_PHILOX, 10)
            ctx.set_step(0)
            ctx.update_many(order)
            s_, n_ = ctx.epoch_elbo()
            out[fork, use_graph] = (s_ / n_, ctx.get_params(), ctx.get_adagrad_state())
            ctx.close()
    for fork in ("1", "0"):
        a, b = out[fork, True], out[fork, False]
        assert a[0] == b[0] and np.array_equal(a[1], b[1]) and np.array_equal(a[2], b[2])
    u = out["0", True]
    for fork in ("1",):
        f = out[fork, True]
        assert abs(f[0] - u[0]) <= 1e-6 * abs(u[0])
        assert np.abs(f[1] - u[1]).max() <= 1e-6 and np.abs(f[2] - u[2]).max() <= 1e-6 * max(1.0, np.abs(u[2]).max())


def arena_split(flat, cfg):
    """The flat arena in reference order as the oracle's named tensors."""
    out, o = {}, 0
    for name, p in zip(cfg.names, O.init_params(cfg)):
        out[name] = flat[o:o + p.size]
        o += p.size
    return out


def one_step_grads(monkeypatch, env, cfg, B, x):
    """keep_grads: the data gradient of ONE Philox step from theta_0 (no earlier Adagrad steps
    to blur a difference), per arena tensor, and the step's SGVB / B."""
    from vaeb_amd import _lib
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    ctx = _lib.Context(cfg.D, cfg.H, cfg.Z, B, decoder=int(cfg.continuous), max_eval_rows=B, dtype=_lib.DTYPE_BF16,
                       keep_grads=True)
    ctx.set_data(x)
    ctx.set_params(O.flatten(O.init_params(cfg)))
    ctx.set_eps_mode(_lib.EPS_PHILOX, 10)
    ctx.set_step(0)
    ctx.update_many(np.array([1], np.int32))
    s_, n_ = ctx.epoch_elbo()
    g = ctx.get_grads()
    ctx.close()
    return s_ / n_, arena_split(g, cfg)


@pytest.mark.parametrize("var,alt,base,Z", [("VAEB_BF_DTT", "0", "1", 40), ("VAEB_BF_DZFUSE", "0", "1", 32),
                                            ("VAEB_BF_DZFUSE", "0", "1", 128), ("VAEB_BF_FORK", "0", "1", 32)])
def test_bf16_tile_form_switches_agree(monkeypatch, var, alt, base, Z):
    """Two forms of the same products (compared on something the gradient moves):
      * VAEB_BF_DTT=0: dhd and dh on A W (EpiDTanh) against the transposed products
        (EpiDTanhT, the default) -- their bias column sums in another order;
      * VAEB_BF_DZFUSE=0: dz + latent backward on the thin launch (Z = 128) or the split-K dz
        GEMM (Z = 32) against dZ as split-K slabs from the forked dhd blocks (EpiDTanhTDz, the
        default; Z % 16 == 0) -- dZ from the bf16-stored dA1 in 256-deep slices;
      * VAEB_BF_FORK=0: the whole default forked step (dz fused into the transposed dhd, dW2 |
        dW6, dW1, dW4 | dW5 on the second stream) against the single-stream step (dhd and dW2
        in one grid on A W, dz as its own product): dA1, dZ and [dMu | dLv] reach every gradient.
    One step's data gradients (keep_grads) agree per tensor to 1e-3 norm-wise (a different fp32
    order can flip a bf16 rounding of dZ or [dMu | dLv]; a broken form is off by O(1)) and the
    ELBO to 1e-6; over 6 Philox steps the Adagrad accumulators (sums of g^2) agree to 1e-3
    relative and the ELBO to 1e-5; graph replay and eager launches are bitwise equal per form."""
    from vaeb_amd import _lib
    cfg = O.Config(D=512, H=264, Z=Z)
    B = 520
    x = (np.random.default_rng(6).random((4 * B, cfg.D)) < 0.4).astype(np.float32)
    order = np.array([1, 3, 0, 2, 3, 1], np.int32)
    out = {}
    for v in (alt, base):
        for use_graph in (True, False):
            monkeypatch.setenv(var, v)
            ctx = _lib.Context(cfg.D, cfg.H, cfg.Z, B, max_eval_rows=B, dtype=_lib.DTYPE_BF16, use_graph=use_graph)
            ctx.set_data(x)
            ctx.set_params(O.flatten(O.init_params(cfg)))
            ctx.set_eps_mode(_lib.EPS_PHILOX, 10)
            ctx.set_step(0)
            ctx.update_many(order)
            s_, n_ = ctx.epoch_elbo()
            out[v, use_graph] = (s_ / n_, ctx.get_params(), ctx.get_adagrad_state())
            ctx.close()
    monkeypatch.setenv(var, base)
    for v in (alt, base):
        a, b = out[v, True], out[v, False]
        assert a[0] == b[0] and np.array_equal(a[1], b[1]) and np.array_equal(a[2], b[2])
    f, u = out[alt, True], out[base, True]
    assert abs(f[0] - u[0]) <= 1e-5 * abs(u[0]), (f[0], u[0])
    assert np.abs(f[1] - u[1]).max() <= 2 * len(order) * cfg.lr
    assert rel(f[2], u[2]) <= 1e-3, rel(f[2], u[2])
    # one step from theta_0: the gradients themselves
    ea, ga = one_step_grads(monkeypatch, {var: alt}, cfg, B, x)
    eb, gb = one_step_grads(monkeypatch, {var: base}, cfg, B, x)
    monkeypatch.setenv(var, base)
    assert abs(ea - eb) <= 1e-6 * abs(eb), (ea, eb)
    bad = {k: rel(ga[k], gb[k]) for k in gb if rel(ga[k], gb[k]) > 1e-3}
    assert not bad, bad


def test_bf16_thin_and_split_k_latent_agree(monkeypatch):
    """The fused thin launches (VAEB_BF_THIN=3 default: heads + latent forward and dz +
    latent backward each one full-K block per 64 / 32 rows) against the split-K slab
    products + latent kernels (=0; =2: dz only), 6 Philox steps at Z = 128: the same sums in a different
    fp32 order, so the ELBO agrees to 1e-5 and the parameters to a few Adagrad steps where
    a bf16 rounding of z or [dMu | dLv] flips; graph replay and eager launches agree bitwise."""
    from vaeb_amd import _lib
    cfg = O.Config(D=512, H=256, Z=128)
    B = 512
    x = (np.random.default_rng(6).random((6 * B, cfg.D)) < 0.4).astype(np.float32)
    order = np.array([3, 1, 4, 1, 5, 0], np.int32)
    out = {}
    for thin in ("3", "2", "0"):   # mask: 1 heads, 2 dz on the thin launches
        for use_graph in (True, False):
            monkeypatch.setenv("VAEB_BF_THIN", thin)
            ctx = _lib.Context(cfg.D, cfg.H, cfg.Z, B, max_eval_rows=B, dtype=_lib.DTYPE_BF16, use_graph=use_graph)
            ctx.set_data(x)
            ctx.set_params(O.flatten(O.init_params(cfg)))
            ctx.set_eps_mode(_lib.EPS_PHILOX, 10)
            ctx.set_step(0)
            ctx.update_many(order)
            s_, n_ = ctx.epoch_elbo()
            out[thin, use_graph] = (s_ / n_, ctx.get_params())
            ctx.close()
    for thin in ("3", "2", "0"):
        a, b = out[thin, True], out[thin, False]
        assert a[0] == b[0] and np.array_equal(a[1], b[1])
    u = out["0", True]
    for thin in ("3", "2"):
        t = out[thin, True]
        assert abs(t[0] - u[0]) <= 1e-5 * abs(u[0]), (thin, t[0], u[0])
        assert np.abs(t[1] - u[1]).max() <= 2 * len(order) * cfg.lr


def test_bf16_gemm8_step_matches_ring_step(monkeypatch):
    """The step with its 256 x 256 launches on the 8-phase loop (VAEB_BF_GEMM8=1; the forked
    dW2 | dW6 and dW3 use them at any size) against the BK = 32 ring: both accumulate every
    output over K in the same 32-wide order, so 6 Philox steps agree to 1e-6."""
    from vaeb_amd import _lib
    cfg = O.Config(D=512, H=256, Z=32)
    B = 512
    x = (np.random.default_rng(5).random((6 * B, cfg.D)) < 0.4).astype(np.float32)
    order = np.array([3, 1, 4, 1, 5, 0], np.int32)
    out = {}
    for g8 in ("0", "1"):
        monkeypatch.setenv("VAEB_BF_GEMM8", "15" if g8 == "1" else "0")
        ctx = _lib.Context(cfg.D, cfg.H, cfg.Z, B, max_eval_rows=B, dtype=_lib.DTYPE_BF16)
        ctx.set_data(x)
        ctx.set_params(O.flatten(O.init_params(cfg)))
        ctx.set_eps_mode(_lib.EPS_PHILOX, 10)
        ctx.set_step(0)
        ctx.update_many(order)
        s_, n_ = ctx.epoch_elbo()
        out[g8] = (s_ / n_, ctx.get_params())
        ctx.close()
    monkeypatch.setenv("VAEB_BF_GEMM8", "0")
    assert abs(out["0"][0] - out["1"][0]) <= 1e-6 * abs(out["0"][0])
    assert np.abs(out["0"][1] - out["1"][1]).max() <= 1e-6


@pytest.mark.parametrize("ako,bko", [(1, 1), (0, 0), (0, 1)])
@pytest.mark.parametrize("M,N,K", [(512, 512, 4096), (296, 520, 328), (768, 256, 1000), (200, 136, 64)])
def test_gemm8_two_slices_combined_in_launch(gctx, ako, bko, M, N, K):
    """Two K slices of every 256 x 256 tile combined inside the launch (split2_combine: the
    first slice to finish publishes its fp32 partial, the second adds it and runs the
    epilogue): partial tiles, K tails and an empty second slice (K = 64), same bound as the
    other GEMM tests; the library also checks that every ticket is back at zero."""
    rng = np.random.default_rng(7 * M + 3 * N + K + 10 * ako + 20 * bko)
    A = rng.standard_normal((M, K)).astype(np.float32)
    B = rng.standard_normal((K, N)).astype(np.float32)
    As = A.T.copy() if ako else A
    Bs = B if bko else B.T.copy()
    C = gctx.test_gemm_bf16(As, Bs, ako, bko, M, N, K, -22)
    Aq = O.bf16_round(A).astype(np.float64)
    Bq = O.bf16_round(B).astype(np.float64)
    ref = Aq @ Bq
    bound = 1e-5 * (np.abs(Aq) @ np.abs(Bq)) + 1e-30
    assert np.all(np.abs(C - ref) <= bound), float(np.max(np.abs(C - ref) / bound))
    assert np.array_equal(C, gctx.test_gemm_bf16(As, Bs, ako, bko, M, N, K, -22))
