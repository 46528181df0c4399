"""Static reader for the reference's pickle-stream files (.mdl checkpoints, modelFrey.pkl,
freyfaces.pkl, mnist.pkl.gz).

NOTHING from the file is ever executed: this module walks the pickle opcode stream itself
(protocols 0-2, the formats Python 2.7 / Theano wrote), builds inert Python literals, and
records GLOBAL / REDUCE / BUILD as plain tuples.  Only one fixed shape of structure is then
turned into data -- numpy's ndarray reconstruction
    REDUCE(numpy.core.multiarray._reconstruct, (numpy.ndarray, (0,), 'b')) + BUILD(
        (1, shape, dtype, fortran, raw_bytes))
with dtype = REDUCE(numpy.dtype, (code, 0, 1)) + BUILD((3, endian, ...)).  Everything else
(RandomState, Theano wrappers such as CudaNdarray_unpickler / TensorSharedVariable) stays
an inert record, and is unwrapped by shape where a known array is inside.
References: VAEB.save / VAEB.load (/root/reference/VAEB.py:189-242), freyFace.py:50-80.
"""
from __future__ import annotations

import codecs
import gzip
import io
import struct

import numpy as np


class Global(tuple):
    """('module', 'name') of a GLOBAL opcode -- never imported."""


class Reduce:
    def __init__(self, func, args):
        self.func, self.args, self.state = func, args, None

    def __repr__(self):
        return f"Reduce({self.func!r}, state={'set' if self.state is not None else None})"


class _Mark:
    pass


_MARK = _Mark()


def _read_line(f):
    line = f.readline()
    if not line.endswith(b"\n"):
        raise ValueError("truncated pickle line")
    return line[:-1]


def _decode_str0(raw: bytes) -> bytes:
    # protocol-0 STRING: a Python-2 repr (quoted, backslash-escaped) of a byte string
    if len(raw) >= 2 and raw[:1] == raw[-1:] and raw[:1] in (b"'", b'"'):
        raw = raw[1:-1]
    return codecs.escape_decode(raw)[0]


def _as_text(b):
    return b.decode("latin1") if isinstance(b, (bytes, bytearray)) else b


def load_frames(data: bytes, max_frames=None):
    """Decode every pickle frame of a byte stream into inert objects."""
    f = io.BytesIO(data)
    frames = []
    while f.tell() < len(data) and (max_frames is None or len(frames) < max_frames):
        frames.append(_load_one(f))
    return frames


def _load_one(f):
    stack, memo = [], {}

    def pop_mark():
        items = []
        while True:
            v = stack.pop()
            if v is _MARK:
                break
            items.append(v)
        items.reverse()
        return items

    while True:
        op = f.read(1)
        if not op:
            raise ValueError("pickle stream ended without STOP")
        c = op
        if c == b".":  # STOP
            return stack.pop()
        elif c == b"(":
            stack.append(_MARK)
        elif c == b"I":
            s = _read_line(f)
            stack.append(True if s == b"01" else False if s == b"00" else int(s))
        elif c == b"L":
            stack.append(int(_read_line(f).rstrip(b"L")))
        elif c == b"F":
            stack.append(float(_read_line(f)))
        elif c == b"S":
            stack.append(_decode_str0(_read_line(f)))
        elif c == b"V":
            stack.append(_read_line(f).decode("raw_unicode_escape"))
        elif c == b"N":
            stack.append(None)
        elif c == b"\x88":
            stack.append(True)
        elif c == b"\x89":
            stack.append(False)
        elif c == b"J":
            stack.append(struct.unpack("<i", f.read(4))[0])
        elif c == b"K":
            stack.append(f.read(1)[0])
        elif c == b"M":
            stack.append(struct.unpack("<H", f.read(2))[0])
        elif c == b"\x8a":  # LONG1
            n = f.read(1)[0]
            stack.append(int.from_bytes(f.read(n), "little", signed=True))
        elif c == b"G":
            stack.append(struct.unpack(">d", f.read(8))[0])
        elif c == b"T":
            n = struct.unpack("<i", f.read(4))[0]
            stack.append(f.read(n))
        elif c == b"U":
            n = f.read(1)[0]
            stack.append(f.read(n))
        elif c == b"X":
            n = struct.unpack("<I", f.read(4))[0]
            stack.append(f.read(n).decode("utf-8"))
        elif c == b"t":
            stack.append(tuple(pop_mark()))
        elif c == b")":
            stack.append(())
        elif c == b"\x85":
            stack.append((stack.pop(),))
        elif c == b"\x86":
            b_ = stack.pop(); a_ = stack.pop(); stack.append((a_, b_))
        elif c == b"\x87":
            c_ = stack.pop(); b_ = stack.pop(); a_ = stack.pop(); stack.append((a_, b_, c_))
        elif c == b"l":
            stack.append(list(pop_mark()))
        elif c == b"]":
            stack.append([])
        elif c == b"a":
            v = stack.pop(); stack[-1].append(v)
        elif c == b"e":
            items = pop_mark(); stack[-1].extend(items)
        elif c == b"d":
            items = pop_mark(); stack.append({items[i]: items[i + 1] for i in range(0, len(items), 2)})
        elif c == b"}":
            stack.append({})
        elif c == b"s":
            v = stack.pop(); k = stack.pop(); stack[-1][k] = v
        elif c == b"u":
            items = pop_mark()
            for i in range(0, len(items), 2):
                stack[-1][items[i]] = items[i + 1]
        elif c == b"c":
            mod = _read_line(f).decode("latin1")
            name = _read_line(f).decode("latin1")
            stack.append(Global((mod, name)))
        elif c == b"R":
            args = stack.pop(); func = stack.pop(); stack.append(Reduce(func, args))
        elif c == b"i":  # INST (protocol 0): recorded, never instantiated
            mod = _read_line(f).decode("latin1")
            name = _read_line(f).decode("latin1")
            stack.append(Reduce(Global((mod, name)), tuple(pop_mark())))
        elif c == b"o":  # OBJ
            items = pop_mark()
            stack.append(Reduce(items[0], tuple(items[1:])))
        elif c == b"\x81":  # NEWOBJ
            args = stack.pop(); cls = stack.pop(); stack.append(Reduce(cls, args))
        elif c == b"b":
            state = stack.pop(); obj = stack[-1]
            if isinstance(obj, Reduce):
                obj.state = state
            else:
                stack[-1] = ("built", obj, state)
        elif c == b"p":
            memo[int(_read_line(f))] = stack[-1]
        elif c == b"q":
            memo[f.read(1)[0]] = stack[-1]
        elif c == b"r":
            memo[struct.unpack("<I", f.read(4))[0]] = stack[-1]
        elif c == b"g":
            stack.append(memo[int(_read_line(f))])
        elif c == b"h":
            stack.append(memo[f.read(1)[0]])
        elif c == b"j":
            stack.append(memo[struct.unpack("<I", f.read(4))[0]])
        elif c == b"\x80":  # PROTO
            f.read(1)
        elif c == b"0":
            stack.pop()
        elif c == b"2":
            stack.append(stack[-1])
        else:
            raise ValueError(f"unsupported pickle opcode {c!r} at offset {f.tell() - 1}")


def _dtype_of(obj):
    if isinstance(obj, Reduce) and obj.func == ("numpy", "dtype"):
        code = _as_text(obj.args[0])
        endian = "<"
        if isinstance(obj.state, tuple) and len(obj.state) > 1 and isinstance(obj.state[1], (str, bytes)):
            endian = _as_text(obj.state[1])
            endian = "<" if endian in ("|", "=") else endian
        return np.dtype(endian + code if code[0] not in "<>|=" else code)
    return None


_RECONSTRUCT = {("numpy.core.multiarray", "_reconstruct"), ("numpy._core.multiarray", "_reconstruct")}


def _as_bytes(raw):
    # protocol-2 pickles written by Python 3 carry bytes as _codecs.encode(text, 'latin1');
    # that one pattern is decoded here as data (nothing is called).
    if isinstance(raw, Reduce) and raw.func == ("_codecs", "encode") and len(raw.args) == 2 \
            and raw.args[1] == "latin1" and isinstance(raw.args[0], str):
        return raw.args[0].encode("latin1")
    if isinstance(raw, str):
        return raw.encode("latin1")
    return raw


def to_array(obj):
    """Turn the inert ndarray-reconstruct record into a numpy array (None if not one)."""
    if not isinstance(obj, Reduce):
        return None
    if obj.func in _RECONSTRUCT and obj.state is not None:
        st = obj.state
        shape, dt, fortran, raw = st[1], _dtype_of(st[2]), st[3], _as_bytes(st[4])
        if dt is None or not isinstance(raw, (bytes, bytearray)):
            return None
        arr = np.frombuffer(bytes(raw), dtype=dt).copy()
        return arr.reshape(shape, order="F" if fortran else "C")
    return None


def find_arrays(obj, depth=0):
    """Depth-first list of every ndarray record inside an inert object."""
    a = to_array(obj)
    if a is not None:
        return [a]
    if depth > 50:
        return []
    out = []
    if isinstance(obj, Reduce):
        out += find_arrays(obj.args, depth + 1)
        out += find_arrays(obj.state, depth + 1)
    elif isinstance(obj, (list, tuple)):
        for v in obj:
            out += find_arrays(v, depth + 1)
    elif isinstance(obj, dict):
        for v in obj.values():
            out += find_arrays(v, depth + 1)
    return out


def _is_randomstate(fr):
    return isinstance(fr, Reduce) and fr.func in (("numpy.random", "__RandomState_ctor"),
                                                  ("numpy.random._pickle", "__randomstate_ctor"))


def read_mdl(path):
    """VAEB .mdl checkpoint (VAEB.save, VAEB.py:189-203): header frames then one frame
    per parameter.  Accepts the 8-field header written by the current save and the
    9-field header VAEB.load expects (VAEB.py:210-218).  Returns (header dict, [arrays])."""
    with open(path, "rb") as fh:
        frames = load_frames(fh.read())
    names = ["n_hidden_units", "n_latent", "continuous", "learning_rate", "batch_size", "prng", "sigmaInit", "L",
             "genericEstimator"]
    hdr_vals, params = [], []
    for fr in frames:
        if not params and (_is_randomstate(fr) or not find_arrays(fr)):
            hdr_vals.append("RandomState" if _is_randomstate(fr) else fr)
            continue
        arrs = [a for a in find_arrays(fr) if a.dtype.kind == "f"]
        if not arrs:
            raise ValueError(f"parameter frame without a float array in {path}")
        params.append(arrs[0])
    return dict(zip(names, hdr_vals)), params


def read_array_pickle(path):
    """A pickled ndarray / tuple of ndarrays (freyfaces.pkl, mnist.pkl.gz, modelFrey.pkl)."""
    opener = gzip.open if str(path).endswith(".gz") else open
    with opener(path, "rb") as fh:
        return read_array_pickle_bytes(fh.read())


def read_array_pickle_bytes(data: bytes):
    """read_array_pickle on an in-memory pickle stream."""
    obj = load_frames(data, max_frames=1)[0]

    def conv(o):
        a = to_array(o)
        if a is not None:
            return a
        if isinstance(o, (list, tuple)):
            return type(o)(conv(v) for v in o)
        return o
    return conv(obj)
