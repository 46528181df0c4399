#!/usr/bin/env python3
"""Per-launch HBM traffic of the MNIST 784-500-20 step (B = 100, fp32) against the
algorithmic bytes of each launch: counters from the committed PMC passes
(profiles/<round>/pmc_mnist_per_launch.json: FETCH_SIZE x 2 + WRITE_SIZE, the guide's gfx950
correction), algorithmic = every operand byte a launch must read plus every byte it must write,
once (DESIGN.md 4.1 lists what each launch computes).

Usage: traffic_ratios.py [profiles/r4/pmc_mnist_per_launch.json]
"""
import json
import os
import sys

D, H, Z, B = 784, 500, 20, 100
Bp = 112                       # rows padded to 16
F = 4                          # fp32
nrb = Bp // 16                 # row blocks
W3, W45, W1, W2 = D * H, 2 * H * Z, Z * H, H * D
b3, b45, b1, b2 = H, 2 * Z, H, D
slab_ml = nrb * (H // 32 + (H % 32 > 0)) * 2 * Z * 16    # encoder [mu | lv] slabs (two h tiles each)
slab_dz = nrb * (H // 16 + (H % 16 > 0)) * Z * 16        # dhd partial dZ slabs

ENC = F * (B * D + W3 + b3 + W45 + b45) + F * (Bp * H + slab_ml)
DW2 = F * (Bp * H + Bp * D) + F * 4 * (W2 + b2)      # hd, dA2 read; theta / Adagrad state read + written
ALG = {   # bytes read + bytes written, each once (round-4 launches; keys match the kernel symbols)
    # encoder (+ the previous step's deferred dW2 | b2 with prior + Adagrad)
    "enc_latent16_w2": ENC + DW2,
    "decout_z": F * (slab_ml + W1 + b1 + W2 + b2 + B * D + b45) + F * (Bp * H + Bp * D + 4 * Bp * Z + Bp * 49),
    # dhd tiles + their partial dZ slabs (the latent backward moved to the last launch)
    "dhd_dz_wgrad": F * (Bp * D + W2 + Bp * H + W1) + F * (Bp * H + slab_dz),
    # reducers (slabs, mu, lv, eps -> [dMu | dLv]), dW3 | b3 (dA3 formed in-workgroup from [dMu | dLv],
    # W4 | W5, h), dW45, dW1 with Adagrad, the ELBO
    "wgrad3": F * (slab_dz + 3 * Bp * Z) + F * 2 * Bp * Z
              + F * (B * D + 2 * Bp * Z + W45 + Bp * H + Bp * Z + Bp * H)
              + F * 4 * (W3 + b3 + W45 + b45 + W1 + b1),
}


def main():
    path = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(__file__), "..", "profiles", "r4",
                                                                "pmc_mnist_per_launch.json")
    data = json.load(open(path))
    print(f"{'launch':<16} {'counter MB':>11} {'algorithmic MB':>15} {'ratio':>6}")
    for key, alg in ALG.items():
        hits = [v for k, v in data.items() if key in k and "hbm_bytes_per_launch" in v]
        if not hits:
            continue
        hbm = hits[0]["hbm_bytes_per_launch"]
        print(f"{key:<16} {hbm / 1e6:11.2f} {alg / 1e6:15.2f} {hbm / alg:6.2f}")


if __name__ == "__main__":
    main()
