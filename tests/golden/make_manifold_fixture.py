"""Generate tests/golden/frey_manifold.npz from the reference's own Frey-face manifold outputs
(run in the build container, where /root/reference exists; the fixture is committed, the
reference never travels).

freyFace.py (/root/reference/freyFace.py) loads the trained Frey model modelFrey.pkl
(:50-66: a pickled list of the 12 parameter arrays in the order W3, W4, W5, W1, W2, W6, b3,
b4, b5, b1, b2, b6), then for ii, jj in 0..9 decodes z = [Phi^-1((ii + 0.9) / 10),
Phi^-1((jj + 0.9) / 10)] with the compiled `freyFace` function (:173-187, 237-245: mu =
sigmoid(tanh(z W1 + b1) W2 + b2), log_sigma = tanh(z W1 + b1) W6 + b6), draws
face ~ N(mu, exp(log_sigma)^2 I) (:357-361) and saves it as freyFaces/FREY{ii}{jj}.jpg
with VAEBImage.save_image (:367).  The pickle is read by vaeb_amd.pickle_static (nothing in
the file is executed); the jpgs are inverted as in make_recon_fixture.jpg_to_x.

Stored: theta [P] (float32, reference order), z [100, 2] (row 10 ii + jj), faces [100, 560].
"""
import os
import sys

import numpy as np
from scipy.stats import norm

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, HERE)
from make_recon_fixture import jpg_to_x  # noqa: E402
from vaeb_amd import pickle_static  # noqa: E402

REF = "/root/reference"


def main():
    params = pickle_static.read_array_pickle(os.path.join(REF, "modelFrey.pkl"))
    shapes = [p.shape for p in params]
    assert shapes[0] == (560, 200) and shapes[3] == (2, 200) and len(params) == 12, shapes
    grid = np.array([norm.ppf((i + 0.9) / 10.0) for i in range(10)])
    z = np.array([[grid[ii], grid[jj]] for ii in range(10) for jj in range(10)], np.float32)
    faces = np.stack([jpg_to_x(os.path.join(REF, "freyFaces", f"FREY{ii}{jj}.jpg"))
                      for ii in range(10) for jj in range(10)])
    theta = np.concatenate([np.asarray(p, np.float32).ravel() for p in params])
    np.savez_compressed(os.path.join(HERE, "frey_manifold.npz"), theta=theta, z=z, faces=faces)
    print(f"{theta.size} parameters, z grid {grid.round(4)}, faces {faces.shape}")


if __name__ == "__main__":
    main()
