"""CPU checks of bench.py's accounting (no GPU): the algorithmic FLOP counts of SURVEY
8(d) for the three bench configs, the per-launch FLOP table the roofline divides by, and
the CPU-baseline leg on a tiny budget."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


@pytest.mark.parametrize("D,H,Z,B,gauss,want", [
    (784, 500, 20, 100, False, 4.100e8),      # MNIST-20: 4.10 MFLOP / image
    (560, 200, 2, 100, True, 1.799e8),        # Frey-2
    (4096, 2048, 128, 8192, False, 7.258e11),  # config 5
])
def test_step_flops_match_survey(D, H, Z, B, gauss, want):
    assert abs(bench.step_flops(D, H, Z, B, gaussian=gauss) - want) <= 1e-3 * want


def test_fused_launch_flops_sum_to_step():
    """The fp32 engine's five launches (folded latent, hfuse groups) cover the step."""
    for gauss in (False, True):
        fl = bench.phase_flops(784, 500, 20, 100, gaussian=gauss)
        parts = ["p1_enc_latent", "p4_decout_z", "p5_dhd_w2", "p67_dz_dh_w1", "p8_wgrad_w3w45"]
        assert sum(fl[k] for k in parts) == bench.step_flops(784, 500, 20, 100, gaussian=gauss)


def test_bf16_launch_flops_sum_to_step():
    fl = bench.phase_flops(4096, 2048, 128, 8192)
    parts = ["bf_enc", "bf_heads", "bf_dechid", "bf_decout", "bf_dhd", "bf_dW26", "bf_dz", "bf_dW1", "bf_dh",
             "bf_dW45", "bf_dW3"]
    assert sum(fl[k] for k in parts) == bench.step_flops(4096, 2048, 128, 8192)


@pytest.mark.parametrize("continuous", [False, True])
def test_cpu_baseline_leg_runs(continuous):
    from oracle import vaeb_oracle as O
    x = O.synthetic_frey(n=40, D=56) if continuous else O.synthetic_mnist(n=40, D=56)
    r = bench.cpu_baseline(56, 20, 2, 10, x, budget_s=0.2, max_steps=5, continuous=continuous)
    assert r["kind"] == "port" and r["value"] > 0 and r["cores"] >= 1
    assert np.isfinite(r["value"])


def test_configs_name_their_metric():
    for name, c in bench.CONFIGS.items():
        assert c["metric"] and c["workload"] and c["dtype"] in ("f32", "bf16")
    assert bench.CONFIGS["mnist"]["metric"] == "SGVB training images/sec + ELBO at MNIST 784-500-20, batch 100"


def test_cpu_baseline_fv_leg_runs():
    from oracle import vaeb_oracle as O
    x = O.synthetic_mnist(n=40, D=56)
    r = bench.cpu_baseline_fv(56, 20, 4, 10, x, budget_s=0.2, max_steps=3)
    assert r["kind"] == "port" and r["value"] > 0


def test_cpu_baseline_fvs_leg_runs():
    from oracle import vaeb_oracle as O
    x = O.synthetic_mnist(n=40, D=56)
    r = bench.cpu_baseline_fv(56, 20, 4, 10, x, budget_s=0.2, max_steps=3, sample=True)
    assert r["kind"] == "port" and r["value"] > 0 and "FVS" in r["sample"]
