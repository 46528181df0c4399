"""vaeb_amd -- MI355X-native (gfx950) implementation of budzianowski/VAEB's SGVB
training step.  The compute path is libvaeb_hip.so (hand-written HIP kernels behind the
C ABI in include/vaeb_hip.h); this package is the host-side mirror of the reference's
VAEB.py interface (VAEB class, args dict, CLI)."""

__version__ = "0.1.0"
