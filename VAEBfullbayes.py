#!/usr/bin/env python3
"""Drop-in entry point for the reference's VAEBfullbayes.py (/root/reference/VAEBfullbayes.py):
`from VAEBfullbayes import VAE` and `python VAEBfullbayes.py` (its __main__, :203-244) on the
MI355X implementation in vaeb_amd/ (vaeb_amd/fullbayes.py)."""
from vaeb_amd.fullbayes import VAE, initial_params_fullbayes, main  # noqa: F401

if __name__ == '__main__':
    main()
