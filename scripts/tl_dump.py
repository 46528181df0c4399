"""Diagnostics: raw per-workgroup stage stamps (VAEB_TIMELINE build) of eager MNIST
784-500-20 steps, saved for offline analysis (gpurun_out/tl_<tag>.npz: [rep][launch][wg][slot],
100 MHz s_memrealtime ticks).  Also records each workgroup's XCC id where the build stamps it."""
import os
import sys

os.environ.setdefault("VAEB_LIB_VARIANT", "tl")
import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import vaeb_oracle as O  # noqa: E402
from vaeb_amd import _lib  # noqa: E402

tag = sys.argv[1] if len(sys.argv) > 1 else "mnist"
D, H, Z, B = (560, 200, 2, 100) if tag.startswith("frey") else (784, 500, 20, 100)
cont = tag.startswith("frey")
x = O.synthetic_frey(n=2000, D=D) if cont else O.synthetic_mnist(n=2000, D=D)
ctx = _lib.Context(D, H, Z, B, max_eval_rows=1000, use_graph=False, decoder=int(cont))
ctx.set_data(x)
ctx.set_params(O.flatten(O.init_params(O.Config(D=D, H=H, Z=Z, continuous=cont))))
for i in range(30):
    ctx.update(i % 20)
reps = np.stack([ctx.debug_timeline(r) for r in range(5)])
os.makedirs("gpurun_out", exist_ok=True)
np.savez_compressed(f"gpurun_out/tl_{tag}{os.environ.get('TL_SUFFIX', '')}.npz", tl=reps)
print("saved", reps.shape)
