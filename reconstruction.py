#!/usr/bin/env python3
"""Drop-in entry point for the reference's reconstruction.py (/root/reference/reconstruction.py):
reconstructions and MSE.res of the trained reconstruction_res/*.mdl models on the MI355X
implementation in vaeb_amd/ (vaeb_amd/reconstruction.py)."""
from vaeb_amd.reconstruction import (MSE, log_file, main, model_file, reconstruction_test,  # noqa: F401
                                     size_continuous_latent_space)

if __name__ == '__main__':
    main()
