"""Dataset readers on files in the reference's layouts (VAEB.py:541-556):
  * freyfaces.pkl: one pickled ndarray [1965 x 560], split rows [:1500] / [1500:] (:544-549)
  * mnist.pkl.gz : gzip of ((x_train, y_train), (x_valid, y_valid), (x_test, y_test)),
                   50000 / 10000 / 10000 rows in the real file (:553-556)
The blobs themselves are absent from the snapshot (.MISSING_LARGE_BLOBS), so the files are
synthesised here, byte for byte the way Python 2.7's cPickle (protocol 2) writes a numpy
ndarray: GLOBAL numpy.core.multiarray._reconstruct, a dtype REDUCE + BUILD state, and the
raw buffer as a BINSTRING -- the stream vaeb_amd.pickle_static decodes without executing
anything.  Row counts are reduced; the layout is the reference's."""
import gzip
import struct

import numpy as np

from vaeb_amd import cli, pickle_static


def _short(b: bytes) -> bytes:
    return b"U" + bytes([len(b)]) + b


def py2_ndarray(a: np.ndarray) -> bytes:
    """Opcode stream (no PROTO / STOP) of a C-contiguous little-endian ndarray as numpy 1.x
    on Python 2.7 pickles it."""
    a = np.ascontiguousarray(a)
    code = a.dtype.str[1:].encode()                     # e.g. b'f4', b'i8'
    out = b"cnumpy.core.multiarray\n_reconstruct\n"
    out += b"cnumpy\nndarray\n" + b"K\x00\x85" + _short(b"b") + b"\x87R"
    shape = b"".join(b"J" + struct.pack("<i", d) for d in a.shape)
    out += b"(K\x01(" + shape + b"t"                      # (1, shape, dtype, fortran, raw)
    out += b"cnumpy\ndtype\n(" + _short(code) + b"K\x00K\x01tR"
    out += b"(K\x03" + _short(b"<") + b"NNNJ\xff\xff\xff\xffJ\xff\xff\xff\xffK\x00tb"
    raw = a.tobytes()
    out += b"\x89" + b"T" + struct.pack("<i", len(raw)) + raw + b"tb"
    return out


def py2_pickle(obj_stream: bytes) -> bytes:
    return b"\x80\x02" + obj_stream + b"."


def tup(*items: bytes) -> bytes:
    return b"(" + b"".join(items) + b"t"


def test_py2_ndarray_stream_roundtrip():
    a = np.arange(12, dtype=np.float32).reshape(3, 4) / 7
    got = pickle_static.read_array_pickle_bytes(py2_pickle(py2_ndarray(a)))
    assert got.dtype == np.float32 and np.array_equal(got, a)


def test_freyfaces_pkl_reader(tmp_path, monkeypatch):
    rng = np.random.default_rng(0)
    x = rng.random((1965, 560)).astype(np.float32)
    (tmp_path / "freyfaces.pkl").write_bytes(py2_pickle(py2_ndarray(x)))
    monkeypatch.chdir(tmp_path)
    xt, xv = cli.load_dataset(True)
    assert xt.shape == (1500, 560) and xv.shape == (465, 560)
    assert np.array_equal(xt, x[:1500]) and np.array_equal(xv, x[1500:])


def test_frey_float64_file_is_cast_to_float32(tmp_path, monkeypatch):
    x = np.random.default_rng(1).random((1600, 560))      # float64 on disk
    (tmp_path / "freyfaces.pkl").write_bytes(py2_pickle(py2_ndarray(x)))
    monkeypatch.chdir(tmp_path)
    xt, xv = cli.load_dataset(True)
    assert xt.dtype == np.float32 and np.array_equal(xt, x[:1500].astype(np.float32))
    assert xv.shape == (100, 560)


def test_mnist_pkl_gz_reader(tmp_path, monkeypatch):
    rng = np.random.default_rng(2)
    parts = []
    arrays = []
    for n in (50, 20, 10):   # train / valid / test
        x = rng.random((n, 784)).astype(np.float32)
        y = rng.integers(0, 10, n).astype(np.int64)
        arrays.append((x, y))
        parts.append(tup(py2_ndarray(x), py2_ndarray(y)))
    with gzip.open(tmp_path / "mnist.pkl.gz", "wb") as f:
        f.write(py2_pickle(tup(*parts)))
    monkeypatch.chdir(tmp_path)
    xt, xv = cli.load_dataset(False)
    assert xt.dtype == np.float32 and np.array_equal(xt, arrays[0][0])
    assert np.array_equal(xv, arrays[1][0])


def test_reader_never_resolves_globals(tmp_path):
    """A stream naming an arbitrary callable is decoded to an inert record, not called."""
    evil = py2_pickle(b"cos\nsystem\n" + _short(b"echo hi") + b"\x85R")
    obj = pickle_static.load_frames(evil)[0]
    assert isinstance(obj, pickle_static.Reduce) and obj.func == ("os", "system")
