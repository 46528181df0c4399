#!/usr/bin/env python3
"""Drop-in entry point for the reference's freyFace.py (/root/reference/freyFace.py):
`from freyFace import VAE` (update / validate / freyFace(z)) and `python freyFace.py
[-continuous]`, the 10 x 10 latent-manifold driver (:311-369), on the MI355X implementation
in vaeb_amd/ (vaeb_amd/freyface.py)."""
from vaeb_amd.freyface import VAE, command_line_args, command_line_flags, draw_manifold, main, manifold_grid  # noqa: F401

if __name__ == '__main__':
    main()
