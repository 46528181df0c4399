"""The world > 1 device path of the sharded data-parallel optimizer, run rank by rank on ONE GPU.

SURVEY §8(e): the step shards by rows, so the reduced gradient is a sum over ranks and the
reference's simultaneous Adagrad (/root/reference/VAEB.py:426-444, the -1/2 sum theta^2 prior of
:386-390) is elementwise.  The library's sharded form (vaeb_hip.hip dp_reduce_update) reduce-
scatters each arena run, updates this rank's 1/W shard plus the replicated remainders, all-gathers
theta' and (bf16 engine) rewrites the shadow of the shards other ranks updated
(step_bf16.hpp shadow_runs_kernel).  RCCL needs one GPU per rank, so the collectives are
emulated here by host copies (include/vaeb_diag.h vaeb_dp_rank_update) while the KERNELS and
the index plan are the ones a rank runs.  For every rank of W = 2, 3, 8:
  * the rank's launch writes exactly its own range (everything else of the out arena stays
    NaN; the gradient outside its reduce-scatter destinations is NaN and never read);
  * theta' composed from the owners (the all-gather) and the Adagrad state composed as
    dp_gather_acc assembles it equal the replicated update BITWISE;
  * after the emulated all-gather every rank holds that theta', and (bf16) its shadow equals
    bf16_round(theta') on every weight element, foreign shards included;
  * the replicated update is the reference's Adagrad rule (float64, 1e-6 relative).
Both bucket forms of a step are run: A (W2 | W6) then B (the rest), as the overlapped step
issues them, and one bucket over the whole arena.
"""
import numpy as np
import pytest

from oracle import vaeb_oracle as O

pytestmark = pytest.mark.gpu

# (D, H, Z, gaussian, dtype, objective): MNIST 784-500-20 and Frey 560-200-2 on the fp32 engine,
# the bf16 engine at a shape whose runs leave remainders (H = 264, Z = 40), Bernoulli and
# Gaussian ([W2 | W6] interleaved in the shadow), and the mean objective (decay term, A18)
CASES = {
    "mnist_fp32": (784, 500, 20, False, "f32", 0),
    "frey_gauss_fp32": (560, 200, 2, True, "f32", 0),
    "bf16_bern": (512, 264, 40, False, "bf16", 0),
    "bf16_gauss": (512, 264, 40, True, "bf16", 0),
    "fp16_bern": (512, 264, 40, False, "fp16", 0),
    "mnist_fp32_mean_map": (784, 500, 20, False, "f32", 1),
}


def bf16_bits(x):
    """bf16 bits of float32 x, round to nearest even (O.bf16_round, whose low 16 bits are 0)."""
    return (O.bf16_round(np.asarray(x, np.float32)).view(np.uint32) >> 16).astype(np.uint16)


def fp16_bits(x):
    """IEEE binary16 bits of float32 x, round to nearest even."""
    return np.asarray(x, np.float32).astype(np.float16).view(np.uint16)


def run_rank(ctx, world, rank, buckets, gsum, theta0, acc0, thg, n_w):
    ctx.set_params(theta0)
    ctx.set_adagrad_state(acc0)
    for i, b in enumerate(buckets):
        ctx.dp_rank_update(world, rank, b, gsum, thg, finish=(i == len(buckets) - 1))
    th = ctx.get_params()
    ac = ctx.get_adagrad_state()
    sh = ctx.get_shadow(n_w) if n_w else None
    return th, ac, sh


def gathered(parts, plans):
    """What the all-gather (theta') / dp_gather_acc (Adagrad state) assemble: shard k of each run
    from rank k, the replicated remainder from rank 0 (vaeb_hip.hip dp_reduce_update,
    dp_gather_acc)."""
    out = np.full_like(parts[0], np.nan)
    for plan in plans:
        for lo, n, S in plan["runs"]:
            W = len(parts)
            for k in range(W):
                out[lo + k * S: lo + (k + 1) * S] = parts[k][lo + k * S: lo + (k + 1) * S]
            out[lo + W * S: lo + n] = parts[0][lo + W * S: lo + n]
    return out


@pytest.fixture(scope="module", params=list(CASES))
def case(request):
    from vaeb_amd import _lib
    D, H, Z, gauss, dt, obj = CASES[request.param]
    ctx = _lib.Context(D, H, Z, 64, decoder=_lib.DEC_GAUSSIAN if gauss else _lib.DEC_BERNOULLI, objective=obj,
                       max_eval_rows=64, dtype={"f32": _lib.DTYPE_F32, "bf16": _lib.DTYPE_BF16, "fp16": _lib.DTYPE_F16}[dt])
    P = ctx.P
    rng = np.random.default_rng(D + H + Z + 7 * gauss + 3 * obj)
    theta0 = (0.01 * rng.standard_normal(P)).astype(np.float32)
    acc0 = (0.1 * np.abs(rng.standard_normal(P))).astype(np.float32)
    acc0[rng.random(P) < 0.1] = 0.0        # elements at their first step
    gsum = rng.standard_normal(P + 1).astype(np.float32)
    plan_all = _lib.dp_plan(D, H, Z, 1, 0, bucket=2, sharded=False,
                            decoder=_lib.DEC_GAUSSIAN if gauss else _lib.DEC_BERNOULLI)
    n_w = 0
    if dt in ("bf16", "fp16"):
        # the weight elements: the arena before the biases (b3 is the first bias)
        n_w = P - (H + 2 * Z + H + D + (D if gauss else 0))
    yield dict(ctx=ctx, D=D, H=H, Z=Z, gauss=gauss, obj=obj, P=P, theta0=theta0, acc0=acc0, gsum=gsum, n_w=n_w,
               P_plan=plan_all["P"], bits=fp16_bits if dt == "fp16" else bf16_bits)
    ctx.close()


def replicated(case):
    c = case
    return run_rank(c["ctx"], 1, 0, [2], c["gsum"], c["theta0"], c["acc0"], None, c["n_w"])


def test_replicated_update_is_the_reference_adagrad(case):
    c = case
    assert c["P_plan"] == c["P"]
    th, ac, sh = replicated(c)
    t0 = c["theta0"].astype(np.float64)
    lr, eps = 0.01, 1e-6
    prior, decay = (0.0, lr * eps) if c["obj"] == 1 else (1.0, 0.0)   # VAEBfullbayes.py:183-184 vs VAEB.py:386-390
    g = c["gsum"][:c["P"]].astype(np.float64) - prior * t0
    a = c["acc0"].astype(np.float64) + g * g
    want = t0 + lr * g / (np.sqrt(a) + eps) - decay * t0 * t0
    assert np.abs(ac - a).max() <= 1e-6 * np.abs(a).max()
    assert np.all(np.abs(th - want) <= 1e-7 + 2e-6 * np.abs(want)), float(np.abs(th - want).max())
    if sh is not None:
        assert np.array_equal(sh, c["bits"](th[:c["n_w"]]))


@pytest.mark.parametrize("world", [2, 3, 8])
@pytest.mark.parametrize("form", ["A_then_B", "all"])
def test_sharded_ranks_compose_to_the_replicated_update(case, world, form):
    from vaeb_amd import _lib
    c = case
    ctx, P, n_w = c["ctx"], c["P"], c["n_w"]
    dec = _lib.DEC_GAUSSIAN if c["gauss"] else _lib.DEC_BERNOULLI
    buckets = [0, 1] if form == "A_then_B" else [2]
    th_rep, ac_rep, _ = replicated(c)

    # pass 1: every rank's own launch, no all-gather yet
    th1, ac1 = [], []
    for r in range(world):
        plans = [_lib.dp_plan(c["D"], c["H"], c["Z"], world, r, bucket=b, decoder=dec) for b in buckets]
        own = np.zeros(P, bool)
        for pl in plans:
            assert not pl["book"] or pl is plans[-1]
            for lo, n in pl["own"]:
                assert not own[lo:lo + n].any(), "a rank's ranges overlap"
                own[lo:lo + n] = True
        th, ac, _ = run_rank(ctx, world, r, buckets, c["gsum"], c["theta0"], c["acc0"], None, n_w)
        # the rank wrote exactly its range: everything else of the out arena is still NaN, and
        # its Adagrad state changed only there
        assert not np.isnan(th[own]).any()
        assert np.isnan(th[~own]).all()
        assert np.array_equal(ac[~own], c["acc0"][~own])
        assert np.array_equal(th[own], th_rep[own]), "own shard differs from the replicated update"
        assert np.array_equal(ac[own], ac_rep[own])
        th1.append(th)
        ac1.append(ac)
    plans_all = [_lib.dp_plan(c["D"], c["H"], c["Z"], world, 0, bucket=b, decoder=dec) for b in buckets]
    # every element is owned by exactly one rank or replicated on all
    th_g = gathered(th1, plans_all)
    ac_g = gathered(ac1, plans_all)
    assert np.array_equal(th_g, th_rep)
    assert np.array_equal(ac_g, ac_rep)

    # pass 2: with the all-gather (the other ranks' theta' copied in) and the shadow fix
    for r in range(world):
        th, ac, sh = run_rank(ctx, world, r, buckets, c["gsum"], c["theta0"], c["acc0"], th_g, n_w)
        assert np.array_equal(th, th_rep), f"rank {r}: theta' after the all-gather differs"
        if n_w:
            want = c["bits"](th_rep[:n_w])
            bad = np.flatnonzero(sh != want)
            assert bad.size == 0, f"rank {r}: {bad.size} shadow entries differ, first at {bad[:5]}"


def test_rank_update_rejects_bad_arguments(case):
    from vaeb_amd import _lib
    c = case
    with pytest.raises(_lib.VaebError):
        c["ctx"].dp_rank_update(2, 2, 0, c["gsum"])          # rank >= world
    with pytest.raises(_lib.VaebError):
        c["ctx"].dp_rank_update(2, 0, 3, c["gsum"])          # no bucket 3
    with pytest.raises(_lib.VaebError):
        c["ctx"].dp_rank_update(2, 0, 0, c["gsum"][:-1])     # P floats instead of P + 1
