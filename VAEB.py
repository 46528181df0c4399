#!/usr/bin/env python3
"""Drop-in entry point: `python VAEB.py --n_latent 20 ...` runs the reference's CLI
(/root/reference/VAEB.py:601-612) on the MI355X implementation in vaeb_amd/."""
from vaeb_amd.cli import (command_line_args, command_line_flags, get_arg, get_flag, main,  # noqa: F401
                          parse_args, print_args, train_model)
from vaeb_amd.model import VAEB  # noqa: F401

if __name__ == '__main__':
    main()
