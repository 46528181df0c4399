"""Generate tests/golden/fv_frey2.npz from the reference's own output files (run in the
build container, where /root/reference exists; the fixture is committed).

  * mu0: the 12 parameters of reconstruction_res/VAE_continuous_2.mdl (Frey 560-200-2),
    flattened in file order (= the reference order W3,W4,W5,W1,W2,W6,b3,b4,b5,b1,b2,b6),
    decoded with vaeb_amd.pickle_static (a static opcode reader: nothing is executed);
  * trace_L / trace_Lvalid: columns 2 and 3 of full_vb_res/continuous_2.trc, one row per
    epoch (the reference writes each row twice, VAEB.py:583-593);
  * fv_mdl_equal: whether full_vb_res/continuous_2.mdl's parameters are bit-identical to
    mu0 (SURVEY 8(c) pin 2: the literal FV path never updates theta).
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from vaeb_amd import pickle_static  # noqa: E402

REF = "/root/reference"


def main():
    hdr, params = pickle_static.read_mdl(os.path.join(REF, "reconstruction_res/VAE_continuous_2.mdl"))
    _, params_fv = pickle_static.read_mdl(os.path.join(REF, "full_vb_res/continuous_2.mdl"))
    mu0 = np.concatenate([p.ravel() for p in params]).astype(np.float32)
    same = all(np.array_equal(a, b) for a, b in zip(params, params_fv))
    rows = [ln.strip().split(",") for ln in open(os.path.join(REF, "full_vb_res/continuous_2.trc")).read().split("\n")[1:]
            if ln.strip()]
    rows = rows[::2]
    L = np.array([float(r[1]) for r in rows])
    Lv = np.array([float(r[2]) for r in rows])
    shapes = np.array([list(p.shape) + [0] * (2 - p.ndim) for p in params], np.int64)
    np.savez_compressed(os.path.join(HERE, "fv_frey2.npz"), mu0=mu0, shapes=shapes, trace_L=L, trace_Lvalid=Lv,
                        fv_mdl_equal=np.array(same), header_n_hidden=hdr["n_hidden_units"], header_n_latent=hdr["n_latent"])
    print("mu0", mu0.shape, "epochs", len(L), "fv mdl bit-identical:", same)


if __name__ == "__main__":
    main()
