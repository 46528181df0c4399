"""The reference's image drivers on the HIP path, end to end against the reference's own
saved images (fixtures tests/golden/recon_frey.npz and frey_manifold.npz):

* reconstruction.py (vaeb_amd/reconstruction.py): models written as .mdl files from the
  trained reference parameters, run through the driver; the jpgs it writes for the reference's
  8 test inputs match the reference's jpgs of the same (model, num_samples, i) to the
  resolution of two JPEG passes, and MSE.res holds the expected error.
* freyFace.py (vaeb_amd/freyface.py): `python freyFace.py -continuous` with a modelFrey.pkl in
  the working directory (the trained reference parameters, re-pickled here) writes
  FREY{ii}{jj}.jpg faces that match the reference's.
"""
import os
import pickle

import numpy as np
import pytest

from oracle import vaeb_oracle as O

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _jpg(path):
    import sys
    sys.path.insert(0, GOLD)
    from make_recon_fixture import jpg_to_x
    return jpg_to_x(path)


def test_reconstruction_driver_matches_reference_images(tmp_path):
    from vaeb_amd import reconstruction as R
    from vaeb_amd.model import VAEB
    f = np.load(os.path.join(GOLD, "recon_frey.npz"))
    os.makedirs(tmp_path / "reconstruction_res")
    x_test = np.concatenate([f["x_orig_z2"], O.synthetic_frey(n=92, seed=5)]).astype(np.float32)
    x_train = O.synthetic_frey(n=300, seed=6)
    for z in (2, 10, 20):
        cfg = O.Config(D=560, H=200, Z=z, continuous=True)
        m = VAEB(x_train, True, 200, z, 100, 1, 0.01, False, False, params=O.unflatten(f[f"theta_z{z}"], cfg))
        m.save(str(tmp_path / "reconstruction_res" / f"continuous_{z}.mdl"))
        m.close()
    np.random.seed(0)
    res = R.main(root=str(tmp_path), data={"continuous": (x_train, x_test)}, data_types=("continuous",))
    lines = open(tmp_path / "reconstruction_res" / "MSE.res").read().splitlines()
    assert lines[0] == "data_type,latent_size,sample_type,MSE" and len(lines) == 7
    assert [l.split(",")[:3] for l in lines[1:]] == [["continuous", str(z), t] for z in (2, 10, 20)
                                                     for t in ("mean", "sample")]
    for z in (2, 10, 20):
        cfg = O.Config(D=560, H=200, Z=z, continuous=True)
        p = O.unflatten(f[f"theta_z{z}"].astype(np.float64), cfg)
        # the mean MSE's expectation: ||y - x||^2 + sum exp(2 log_sigma) per row
        y, ls = O.reconstruct_full(p, x_test.astype(np.float64), None, cfg)
        e_row = ((y - x_test) ** 2).sum(1) + np.exp(2 * ls).sum(1)
        assert abs(res[("continuous", z)][0] - e_row.mean()) < 5 * e_row.std() / np.sqrt(len(x_test)) + 0.05
        for ns, key in ((0, "y_sample"), (20, "y_sample20")):
            ours = np.stack([_jpg(str(tmp_path / "reconstruction_res" / f"continuous_{z}__image_{ns}_{i}_sample.jpg"))
                             for i in range(8)])
            ref = f[f"{key}_z{z}"]
            d_own = np.abs(ours - ref).mean()
            d = np.abs(ours[:, None, :] - ref[None, :, :]).mean(-1)
            assert d_own <= 0.03, (z, ns, d_own)
            if z >= 10:   # each output nearer its own reference image than others on average
                assert d_own < 0.85 * d[~np.eye(8, dtype=bool)].mean(), (z, ns)
            orig = np.stack([_jpg(str(tmp_path / "reconstruction_res" / f"continuous_{z}__image_{ns}_{i}_original.jpg"))
                             for i in range(8)])
            assert np.abs(orig - f[f"x_orig_z{z}"]).mean() <= 0.02


def test_reconstruction_driver_bernoulli_models_with_mnist_split_data(tmp_path):
    """VAEB.load of a Bernoulli (MNIST) model takes the data as VAEB.py:237-239
    returns it -- ((x, y) train, valid, test) -- whose first element is a ragged pair.
    reconstruction.main loads the discrete models first; each must load, reconstruct and
    log its two MSE lines, the mean reconstruction equal to the oracle's decoder mean."""
    from vaeb_amd import reconstruction as R
    from vaeb_amd.model import VAEB
    os.makedirs(tmp_path / "reconstruction_res")
    x = O.synthetic_mnist(n=400, seed=3)
    lab = np.zeros(100, np.int64)
    data = ((x[:200], np.zeros(200, np.int64)), (x[200:300], lab), (x[300:], lab))
    thetas = {}
    for z in (2, 10, 20):
        cfg = O.Config(D=784, H=500, Z=z)
        rng = np.random.default_rng(z)   # away from the near-constant initial decoder
        thetas[z] = [(a + rng.normal(0, 0.1, a.shape)).astype(np.float32) for a in O.init_params(cfg)]
        m = VAEB(x[:200], False, 500, z, 100, 1, 0.01, False, False, params=thetas[z])
        m.save(str(tmp_path / "reconstruction_res" / f"discrete_{z}.mdl"))
        m.close()
    res = R.main(root=str(tmp_path), data={"discrete": data}, data_types=("discrete",))
    lines = open(tmp_path / "reconstruction_res" / "MSE.res").read().splitlines()
    assert [l.split(",")[:3] for l in lines[1:]] == [["discrete", str(z), t] for z in (2, 10, 20)
                                                     for t in ("mean", "sample")]
    for z in (2, 10, 20):
        cfg = O.Config(D=784, H=500, Z=z)
        y, _ = O.reconstruct_full([p.astype(np.float64) for p in thetas[z]], x[300:].astype(np.float64), None, cfg)
        want = float(np.mean(np.linalg.norm(y - x[300:], axis=1) ** 2))
        assert abs(res[("discrete", z)][0] - want) <= 1e-4 * want, (z, res[("discrete", z)][0], want)
        model, d = VAEB.load(str(tmp_path / "reconstruction_res" / f"discrete_{z}.mdl"), data=data)
        assert model.N == 200 and d is data
        model.close()


def test_freyface_driver_matches_reference_faces(tmp_path, monkeypatch):
    from vaeb_amd import freyface
    m = np.load(os.path.join(GOLD, "frey_manifold.npz"))
    cfg = O.Config(D=560, H=200, Z=2, continuous=True)
    with open(tmp_path / "modelFrey.pkl", "wb") as fh:   # freyFace.py:50-53 reads this list
        pickle.dump([np.asarray(a, np.float32) for a in O.unflatten(m["theta"], cfg)], fh, protocol=2)
    monkeypatch.chdir(tmp_path)
    x = O.synthetic_frey(n=400)
    model = freyface.main(["-continuous", "--n_latent", "2"], data=(x[:300], x[300:]), out_dir="freyFaces",
                          out=lambda *a: None)
    assert np.array_equal(model._ctx.get_params(), m["theta"])   # the pickled model replaced the init
    faces = np.stack([_jpg(str(tmp_path / "freyFaces" / f"FREY{ii}{jj}.jpg")) for ii in range(10) for jj in range(10)])
    d = np.abs(faces - m["faces"]).mean()
    M = np.abs(faces[None, :, :] - m["faces"][:, None, :]).mean(-1)
    assert d <= 0.025 and (M.argmin(1) == np.arange(100)).mean() >= 0.75, d
    mu, ls = model.freyFace(m["z"])
    rm, rl = O.decode(O.unflatten(m["theta"].astype(np.float64), cfg), m["z"].astype(np.float64), cfg)
    assert np.abs(mu - rm).max() <= 1e-5 and np.abs(ls - rl).max() <= 1e-4
    model.close()
