"""Diagnostics: one bf16 step with VAEB_BF_DZFUSE=1 and =0 against the bf16-rounded oracle
(D 512, H, Z, B from argv): the relative error of every data-gradient tensor."""
import os
import sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import vaeb_oracle as O  # noqa: E402

Z, H, B = (int(a) for a in sys.argv[1:4])
cfg = O.Config(D=512, H=H, Z=Z)
x = O.synthetic_mnist(n=3 * B, D=cfg.D)
params = O.init_params(cfg)
rng = np.random.default_rng(5)
params = [p if p.ndim == 2 else (0.01 * rng.standard_normal(p.shape)).astype(np.float32) for p in params]
acc = [np.full_like(p, 1e-3) for p in params]
eps = rng.standard_normal((1, B, cfg.Z)).astype(np.float32)
xb = x[B:2 * B].astype(np.float64)
q_elbo, _, _, q_aux = O.step([p.astype(np.float64) for p in params], [a.astype(np.float64) for a in acc], xb,
                             eps.astype(np.float64), cfg, q=O.bf16_round)
for v in ("1", "0"):
    os.environ["VAEB_BF_DZFUSE"] = v
    from vaeb_amd import _lib
    ctx = _lib.Context(cfg.D, cfg.H, cfg.Z, B, keep_grads=True, max_eval_rows=512, dtype=_lib.DTYPE_BF16)
    ctx.set_data(x)
    ctx.set_params(O.flatten(params))
    ctx.set_adagrad_state(O.flatten(acc))
    ctx.set_eps_mode(1)
    ctx.push_eps(eps)
    e = ctx.update(1)
    g = ctx.get_grads()
    ctx.close()
    errs = []
    for (n, s), gg, rq in zip(O.param_shapes(cfg), O.unflatten(g, cfg), q_aux["data_grads"]):
        errs.append(f"{n} {np.linalg.norm(gg.reshape(s) - rq) / max(np.linalg.norm(rq), 1e-30):.1e}")
    print("DZFUSE", v, "elbo", e, q_elbo, " ".join(errs))
