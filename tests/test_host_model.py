"""Host-side pieces of the drop-in that run without a GPU: parameter layout and init
(restated in vaeb_amd/model.py, must equal the oracle), the static checkpoint reader
(vaeb_amd/pickle_static.py) on files written by vaeb_amd's own writer and -- where the
reference snapshot is present -- on the reference's .mdl / modelFrey.pkl files."""
import os
import pickle

import numpy as np
import pytest

from oracle import vaeb_oracle as O
from vaeb_amd import model, pickle_static

REF = "/root/reference"


@pytest.mark.parametrize("continuous", [False, True])
def test_product_init_equals_oracle_init(continuous):
    D, H, Z = (560, 200, 2) if continuous else (784, 500, 20)
    a = model.initial_params(D, H, Z, continuous)
    b = O.init_params(O.Config(D=D, H=H, Z=Z, continuous=continuous))
    assert [x.shape for x in a] == [x.shape for x in b]
    assert all(np.array_equal(x, y) for x, y in zip(a, b))
    assert [n for n, _ in model.param_shapes(D, H, Z, continuous)] == O.Config(D=D, H=H, Z=Z, continuous=continuous).names


def test_checkpoint_writer_reader_roundtrip(tmp_path):
    """The format VAEB.save writes (9 header frames + one ndarray frame per parameter)."""
    params = model.initial_params(30, 7, 3, True)
    f = tmp_path / "m.mdl"
    with open(f, "wb") as fh:
        for v in (7, 3, True, 0.01, 100, np.random.RandomState(10), 0.01, 1, False):
            pickle.dump(v, fh, protocol=2)
        for p in params:
            pickle.dump(p, fh, protocol=2)
    hdr, got = pickle_static.read_mdl(str(f))
    assert hdr["n_hidden_units"] == 7 and hdr["n_latent"] == 3 and hdr["continuous"] is True
    assert hdr["genericEstimator"] is False and hdr["prng"] == "RandomState"
    assert all(np.array_equal(a, b) for a, b in zip(params, got))


def test_static_reader_never_imports(tmp_path):
    """A GLOBAL naming a callable is recorded, never resolved or called."""
    f = tmp_path / "evil.pkl"
    f.write_bytes(b"cos\nsystem\n(S'echo pwned'\ntR.")
    obj = pickle_static.load_frames(f.read_bytes())[0]
    assert isinstance(obj, pickle_static.Reduce) and obj.func == ("os", "system")


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference snapshot not present")
def test_reads_reference_checkpoints():
    hdr, p = pickle_static.read_mdl(os.path.join(REF, "reconstruction_res/VAE_continuous_2.mdl"))
    assert hdr["n_hidden_units"] == 200 and len(p) == 12 and p[0].shape == (560, 200)
    hdr8, p8 = pickle_static.read_mdl(os.path.join(REF, "full_vb_res/continuous_2.mdl"))
    assert "genericEstimator" not in hdr8  # the 8-field header of the current VAEB.save
    frey = pickle_static.read_array_pickle(os.path.join(REF, "modelFrey.pkl"))
    assert [a.shape for a in frey][:2] == [(560, 200), (200, 2)]


def test_theano_stream_emulation_shapes():
    s = model.TheanoStreamEmulation(L=2)
    e = s.draw(5, 3)
    assert e.shape == (2, 5, 3) and e.dtype == np.float32
    # first op seed as recalled in SURVEY 8(c)
    assert np.random.RandomState(10).randint(2 ** 30) == 91571465
