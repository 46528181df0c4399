"""Host side of the image drivers (no GPU): VAEBImage.save_image's layout, the drivers' argument
tables and the reference-form dataset tuple."""
import os
import sys

import numpy as np

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_save_image_layout_inverts_like_the_reference_jpgs(tmp_path):
    """VAEBImage.py:14-24: a Frey face is written as a 28-row x 20-column jpg (the reference's
    saved images have that size); make_recon_fixture.jpg_to_x inverts it to the JPEG's
    resolution, as it does for the reference's own files."""
    from PIL import Image
    sys.path.insert(0, GOLD)
    from make_recon_fixture import jpg_to_x
    from vaeb_amd.image import save_image
    x = np.load(os.path.join(GOLD, "recon_frey.npz"))["x_orig_z2"][3]
    p = str(tmp_path / "f.jpg")
    save_image(x, p)
    assert Image.open(p).size == (20, 28)
    assert np.abs(jpg_to_x(p) - x).mean() < 0.005
    m = np.linspace(0, 1, 784)
    save_image(m, str(tmp_path / "m.jpg"))
    assert Image.open(str(tmp_path / "m.jpg")).size == (28, 28)


def test_freyface_args_and_grid():
    from vaeb_amd import freyface
    from vaeb_amd.cli import parse_args
    a = parse_args(["-continuous", "--n_latent", "2", "--bogus", "1"], freyface.command_line_args,
                   freyface.command_line_flags, flag_prefix="-")
    assert a["continuous"] is True and a["n_latent"] == 2 and a["n_epochs"] == 2000 and a["hidden_unit"] == -1
    g = freyface.manifold_grid()
    assert g.shape == (100, 2) and np.allclose(g[0], g[0, 0]) and g[99, 0] > 2.3
    f = np.load(os.path.join(GOLD, "frey_manifold.npz"))
    assert np.allclose(g, f["z"], atol=1e-6)


def test_reference_form_mnist_tuple():
    from vaeb_amd.cli import load_dataset
    (xtr, ytr), (xv, yv), (xte, yte) = load_dataset(False, synthetic=True, splits=3)
    assert xtr.shape == (50000, 784) and xv.shape == xte.shape == (10000, 784) and len(ytr) == 50000
