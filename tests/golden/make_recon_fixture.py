"""Generate tests/golden/recon_frey.npz from the reference's own reconstruction outputs (run in
the build container, where /root/reference exists; the fixture is committed, the reference
never travels).

reconstruction.py (/root/reference/reconstruction.py:19-30) loaded the trained Frey models
reconstruction_res/continuous_{2,10,20}.mdl and, for the first 8 test rows x_i, saved
VAEBImage.save_image(x_i) as `..._image_0_{i}_original.jpg` and
VAEBImage.save_image(model.reconstruct(x_i, 0)) as `..._image_0_{i}_sample.jpg`
(num_samples = 0: the decoder mean at z = mu, then the continuous branch's closing
multivariate_normal draw with cov = exp(y_log_sigma)^2 I, VAEB.py:267-297).

save_image (VAEBImage.py:14-22) maps a 560-vector x to pixels as
    X = x.reshape(20, 28, order='F');  img = rotate((1 - X) * 255, -90)   (a 20 x 28 jpg)
so the inverse applied here is
    X = rot90(img, +1) / 255;  x = (1 - X).reshape(-1, order='F')
The JPEG round trip quantises and blurs every pixel (and the sample carries the draw's
noise), so the pin is statistical: tests compare mean |y - y_ref| against the same
statistic for mismatched (input, output) pairs.

The num_samples = 20 pass of the same loop (reconstruction.py:21-34) saved
`..._image_20_{i}_original.jpg` (the same 8 inputs) and `..._image_20_{i}_sample.jpg`:
model.reconstruct(x_i, 20), i.e. the decoder outputs averaged over 20 posterior draws
z = mu + exp(lv / 2) eps (VAEB.py:271-291), then the closing draw.

Stored: for each z in (2, 10, 20): the 12 parameters flattened in file (= reference) order,
x_orig [8, 560], y_sample [8, 560] (num_samples = 0) and y_sample20 [8, 560]
(num_samples = 20) (float32).
"""
import os
import sys

import numpy as np
from PIL import Image

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from vaeb_amd import pickle_static  # noqa: E402

REF = "/root/reference/reconstruction_res"


def jpg_to_x(path):
    """Invert VAEBImage.save_image for a 560-pixel Frey face (grey channel 0 of the RGB jpg)."""
    img = np.asarray(Image.open(path).convert("RGB"), np.float64)[..., 0]   # [28 rows x 20 cols]
    X = np.rot90(img, 1) / 255.0                                             # [20 x 28]
    return (1.0 - X).reshape(-1, order="F").astype(np.float32)


def main():
    out = {}
    for z in (2, 10, 20):
        hdr, params = pickle_static.read_mdl(os.path.join(REF, f"continuous_{z}.mdl"))
        assert int(hdr["n_latent"]) == z and int(hdr["n_hidden_units"]) == 200 and bool(hdr["continuous"])
        out[f"theta_z{z}"] = np.concatenate([p.ravel() for p in params]).astype(np.float32)
        out[f"x_orig_z{z}"] = np.stack([jpg_to_x(os.path.join(REF, f"continuous_{z}__image_0_{i}_original.jpg"))
                                        for i in range(8)])
        out[f"y_sample_z{z}"] = np.stack([jpg_to_x(os.path.join(REF, f"continuous_{z}__image_0_{i}_sample.jpg"))
                                          for i in range(8)])
        x20 = np.stack([jpg_to_x(os.path.join(REF, f"continuous_{z}__image_20_{i}_original.jpg")) for i in range(8)])
        assert np.array_equal(x20, out[f"x_orig_z{z}"]), "both passes save the same 8 inputs"
        out[f"y_sample20_z{z}"] = np.stack([jpg_to_x(os.path.join(REF, f"continuous_{z}__image_20_{i}_sample.jpg"))
                                            for i in range(8)])
        print(f"z={z}: {out[f'theta_z{z}'].size} parameters, header {hdr}")
    np.savez_compressed(os.path.join(HERE, "recon_frey.npz"), **out)


if __name__ == "__main__":
    main()
