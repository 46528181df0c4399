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


def test_folded_launch_flops_sum_to_step():
    """The folded latent backward's four launches (latent.hpp, latent_bwd.hpp) cover the step."""
    for gauss in (False, True):
        fl = bench.phase_flops(784, 500, 20, 100, gaussian=gauss)
        parts = ["p1_enc_latent", "p4_decout_z", "p5_dhd_dz_w2", "p8_wgrad_w3w45w1"]
        assert sum(fl[k] for k in parts) == bench.step_flops(784, 500, 20, 100, gaussian=gauss)
    fl = bench.phase_flops(4096, 2048, 128, 8192)
    assert fl["bf_dhd_dW26"] == fl["bf_dhd"] + fl["bf_dW26"]


def test_deferred_dw2_launch_flops_sum_to_step():
    """Round 4's MNIST form: the previous step's dW2 rides the encoder launch, the dhd launch has
    none; the four launches still cover the step (the roofline divides by these)."""
    for gauss in (False, True):
        fl = bench.phase_flops(784, 500, 20, 100, gaussian=gauss)
        parts = ["p1_enc_latent_w2", "p4_decout_z", "p5_dhd_dz", "p8_wgrad_w3w45w1"]
        assert sum(fl[k] for k in parts) == bench.step_flops(784, 500, 20, 100, gaussian=gauss)


def test_library_launch_names_have_flops_and_symbols():
    """Every profile id the library emits for the fp32 four-launch step has a FLOP count and a
    kernel symbol for the committed PMC lookup (bench.KERNEL_SYMBOLS)."""
    src = open(os.path.join(ROOT, "vaeb_amd", "csrc", "vaeb_hip.hip")).read()
    fl = bench.phase_flops(784, 500, 20, 100)
    for name in ("p1_enc_latent_w2", "p5_dhd_dz", "p8_wgrad_w3w45w1", "p4_decout_z"):
        assert f'"{name}"' in src
        assert name in fl and name in bench.KERNEL_SYMBOLS


def test_round4_traffic_file_resolves_every_launch():
    """bench.py reads roofline.traffic from the committed round-4 PMC passes: each of the four
    MNIST launches resolves to a per-launch byte count there."""
    path = bench.PMC_FILES["mnist"]
    assert os.path.exists(path), path
    for name in ("p1_enc_latent_w2", "p4_decout_z", "p5_dhd_dz", "p8_wgrad_w3w45w1"):
        v = bench.committed_traffic(name, path)
        assert v is not None and v > 1e6, (name, v)


def test_bf16_symbols_resolve_in_the_newest_synth_pmc():
    """every bf16 launch of the profiled (unforked) config-5 step maps to a kernel of
    the newest committed synth PMC file under its current name, and the forms the profiled step
    does not run (the forked dhd, dW2) do not silently take another launch's bytes."""
    path = bench.PMC_FILES["synth"]
    assert os.path.exists(path), path
    import json
    names = list(json.load(open(path)))
    got = {}
    for k in ("bf_enc", "bf_dechid", "bf_heads", "bf_dz", "bf_decout", "bf_dh", "bf_dhd_dW26", "bf_dW3"):
        v = bench.committed_traffic(k, path)
        assert v is not None and v > 1e6, (k, v)
        got[k] = v
    # the current forms are matched first: the 8-phase encoder, the transposed decoder
    def first_match(k):
        sym = bench.KERNEL_SYMBOLS[k]
        for alt in sym:
            for n in names:
                if all(t in n for t in alt):
                    return n
    assert "gemm8_kernel<0, 1," in first_match("bf_enc")
    assert "EpiDecOutT" in first_match("bf_decout")
    assert "gemm_kernel<0, 1, 128," in first_match("bf_dechid")
    assert got["bf_enc"] != got["bf_dechid"]


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
        assert c["metric"] and c["workload"] and c["dtype"] in bench.DTYPES
    assert bench.CONFIGS["mnist"]["metric"] == "SGVB training images/sec + ELBO at MNIST 784-500-20, batch 100"
    # BASELINE.json config 5: "fp16 MFMA"
    assert bench.CONFIGS["synth"]["dtype"] == "fp16" and "fp16 MFMA" in bench.CONFIGS["synth"]["metric"]


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


STUB = r'''
import json, os, sys, time
out = sys.argv[1]
rank = int(os.environ["RANK"])
rec = {k: os.environ.get(k) for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT",
                                      "HSA_ENABLE_IPC_MODE_LEGACY")}
rec["argv"] = sys.argv[1:]
json.dump(rec, open(os.path.join(out, f"rank{rank}.json"), "w"))
if len(sys.argv) > 2 and sys.argv[2] == "fail" and rank == 1:
    sys.exit(3)
if len(sys.argv) > 2 and sys.argv[2] == "fail":
    time.sleep(60)   # a healthy rank waiting in a collective: the launcher must stop it
'''


def test_launcher_spawns_one_process_per_gpu(tmp_path):
    """bench.py --gpus N without WORLD_SIZE: N children, RANK = LOCAL_RANK = r, WORLD_SIZE = N,
    one rendezvous on 127.0.0.1 (the GPU library is never touched by the parent)."""
    stub = tmp_path / "stub.py"
    stub.write_text(STUB)
    rc = bench.spawn_ranks(4, [str(tmp_path)], script=str(stub))
    assert rc == 0
    import json
    recs = [json.load(open(tmp_path / f"rank{r}.json")) for r in range(4)]
    assert [r["RANK"] for r in recs] == ["0", "1", "2", "3"]
    assert [r["LOCAL_RANK"] for r in recs] == ["0", "1", "2", "3"]
    assert all(r["WORLD_SIZE"] == "4" and r["MASTER_ADDR"] == "127.0.0.1" for r in recs)
    assert len({r["MASTER_PORT"] for r in recs}) == 1
    assert all(r["HSA_ENABLE_IPC_MODE_LEGACY"] == "0" for r in recs)


def test_launcher_stops_the_job_when_a_rank_fails(tmp_path):
    import time
    stub = tmp_path / "stub.py"
    stub.write_text(STUB)
    t0 = time.time()
    rc = bench.spawn_ranks(3, [str(tmp_path), "fail"], script=str(stub))
    assert rc == 3 and time.time() - t0 < 30


def test_bench_main_refuses_world_mismatch(monkeypatch):
    monkeypatch.setenv("WORLD_SIZE", "2")
    with pytest.raises(SystemExit):
        bench.main(["--gpus", "4"])
