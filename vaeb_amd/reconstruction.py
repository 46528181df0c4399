"""Drop-in for the reference's reconstruction.py (/root/reference/reconstruction.py:1-61):
for each trained model reconstruction_res/{discrete,continuous}_{2,10,20}.mdl, save 8
original / reconstructed image pairs for num_samples in (0, 20) and append the mean squared
reconstruction error to reconstruction_res/MSE.res.

The reconstructions run in libvaeb_hip.so (VAEB.reconstruct -> vaeb_reconstruct_full: the
encoder, z = mu or 20 posterior draws, the decoder, averaged on device).  The reference's
continuous MSE calls reconstruct once per test row (:14-18); here the whole test set is one
call -- every row still gets its own posterior draws and its own closing
N(y_mu, exp(y_log_sigma)^2 I) draw, so the estimator is the same.
"""
from __future__ import annotations

import os

import numpy as np

from .image import save_image

size_continuous_latent_space = [2, 10, 20]        # reconstruction.py:5
model_file = 'reconstruction_res/{0}_{1}.mdl'     # :6
log_file = 'reconstruction_res/MSE.res'           # :7


def MSE(model, x_test, num_samples):
    """reconstruction.py:9-18: mean over rows of ||reconstruct(x) - x||^2."""
    samples = model.reconstruct(np.asarray(x_test, np.float32), num_samples)
    return float(np.mean(np.linalg.norm(samples - x_test, axis=1) ** 2))


def reconstruction_test(x_test, model, file_prefix, continuous, log=log_file):
    """reconstruction.py:20-42: 8 (original, reconstruction) jpg pairs and one MSE.res line per
    num_samples in (0, 20).  Returns {num_samples: mse}."""
    res = {}
    for num_samples in [0, 20]:
        print('num_samples :\n{0}'.format(num_samples))
        for i in range(8):
            sample = model.reconstruct(x_test[i], num_samples)
            save_image(x_test[i], file_prefix + '_image_{0}_{1}_original.jpg'.format(num_samples, i))
            save_image(sample, file_prefix + '_image_{0}_{1}_sample.jpg'.format(num_samples, i))
        mse = MSE(model, x_test, num_samples)
        with open(log, 'a') as f:
            f.write('{0},{1},{2},{3}\n'.format('continuous' if continuous else 'discrete', model.n_latent,
                                               'mean' if num_samples == 0 else 'sample', mse))
        res[num_samples] = mse
    return res


def main(root='.', data=None, data_types=('discrete', 'continuous'), **kw):
    """reconstruction.py:45-58, with paths under `root`.  data: {data_type: the dataset as
    VAEB.load returns it} overrides freyfaces.pkl / mnist.pkl.gz (tests)."""
    from .model import VAEB
    log = os.path.join(root, log_file)
    with open(log, 'w') as f:
        f.write('data_type,latent_size,sample_type,MSE\n')
    out = {}
    for data_type in data_types:
        for s in size_continuous_latent_space:
            filename = os.path.join(root, model_file.format(data_type, s))
            model, d = VAEB.load(filename, data=None if data is None else data[data_type], **kw)
            if model.continuous:
                (x_train, x_test) = d
            else:
                (x_train, y_train), (x_valid, y_valid), (x_test, y_test) = d
            prefix = os.path.join(root, "reconstruction_res/{0}_{1}_".format(data_type, s))
            out[(data_type, s)] = reconstruction_test(np.asarray(x_test, np.float32), model, prefix,
                                                      model.continuous, log)
            model.close()
    return out
