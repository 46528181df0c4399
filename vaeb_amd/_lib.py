"""ctypes binding of libvaeb_hip.so (include/vaeb_hip.h).

The library is built in-tree (vaeb_amd/libvaeb_hip.so, see __graft_entry__.build()).
There is no CPU fallback: if the shared object is missing or a call fails, an error is
raised.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libvaeb_hip.so")
# diagnostics A/B only: an alternative in-tree build of the same library (scripts/)
if os.environ.get("VAEB_LIB_VARIANT"):
    LIB_PATH = os.path.join(HERE, f"libvaeb_hip_{os.environ['VAEB_LIB_VARIANT']}.so")

DEC_BERNOULLI, DEC_GAUSSIAN = 0, 1
EST_LB, EST_LA, EST_FV, EST_FVS = 0, 1, 2, 3   # FVS: weight-sampling extension (include/vaeb_hip.h)
OBJ_SUM_PRIOR, OBJ_MEAN_MAP = 0, 1
EPS_PHILOX, EPS_HOST = 0, 1
DTYPE_F32, DTYPE_BF16, DTYPE_F16 = 0, 1, 2

# Every symbol declared in include/vaeb_hip.h (the drop-in boundary) and in
# include/vaeb_diag.h (measurement / test hooks); checked by tests/test_abi.py.
EXPORTS = [
    "vaeb_last_error", "vaeb_version", "vaeb_create", "vaeb_destroy", "vaeb_num_params",
    "vaeb_set_data", "vaeb_set_params", "vaeb_get_params", "vaeb_set_adagrad_state",
    "vaeb_get_adagrad_state", "vaeb_set_fv_state", "vaeb_get_fv_state", "vaeb_set_eps_mode",
    "vaeb_push_eps", "vaeb_set_step", "vaeb_get_step", "vaeb_update", "vaeb_update_async", "vaeb_update_many",
    "vaeb_epoch_elbo", "vaeb_synchronize", "vaeb_validate", "vaeb_reconstruct", "vaeb_reconstruct_sampled",
    "vaeb_reconstruct_full", "vaeb_decode",
    "vaeb_comm_unique_id", "vaeb_comm_init", "vaeb_comm_count", "vaeb_set_valid_data", "vaeb_validate_resident",
    "vaeb_checkpoint_save", "vaeb_checkpoint_load", "vaeb_get_grads", "vaeb_get_activation", "vaeb_push_fv_noise",
    "vaeb_ae_create", "vaeb_ae_destroy", "vaeb_ae_num_params", "vaeb_ae_set_data", "vaeb_ae_set_params",
    "vaeb_ae_get_params", "vaeb_ae_set_adagrad_state", "vaeb_ae_get_adagrad_state", "vaeb_ae_train",
    "vaeb_ae_train_many", "vaeb_ae_reconstruct", "vaeb_ae_encode", "vaeb_ae_decode",
]
DIAG_EXPORTS = ["vaeb_profile_steps", "vaeb_kernel_name", "vaeb_debug_timeline", "vaeb_test_gemm_bf16",
                "vaeb_bench_gemm_bf16", "vaeb_graph_status", "vaeb_comm_info", "vaeb_time_update_many", "vaeb_busy",
                "vaeb_dp_plan", "vaeb_dp_rank_update", "vaeb_get_shadow"]
GRAPH_MODES = {0: "off", 1: "not_captured", 2: "replay", 3: "eager_fallback"}
AE_MAX_LAYERS = 8
AE_BINARY, AE_CONT = 0, 1
ACT = {"tanh": 0, "sigmoid": 1, "relu": 2}


class VaebConfig(ctypes.Structure):
    _fields_ = [
        ("D", ctypes.c_int32), ("H", ctypes.c_int32), ("Z", ctypes.c_int32), ("B", ctypes.c_int32),
        ("B_global", ctypes.c_int32), ("row_offset", ctypes.c_int32), ("L", ctypes.c_int32),
        ("decoder", ctypes.c_int32), ("estimator", ctypes.c_int32), ("objective", ctypes.c_int32),
        ("lr", ctypes.c_float), ("adagrad_eps", ctypes.c_float), ("device", ctypes.c_int32),
        ("max_eval_rows", ctypes.c_int32), ("use_graph", ctypes.c_int32), ("keep_grads", ctypes.c_int32),
        ("dtype", ctypes.c_int32), ("reserved", ctypes.c_int32 * 5),
    ]


class AEConfigC(ctypes.Structure):
    _fields_ = [
        ("Dobs", ctypes.c_int32), ("n_enc", ctypes.c_int32), ("Denc", ctypes.c_int32 * 8),
        ("Dz", ctypes.c_int32), ("n_dec", ctypes.c_int32), ("Ddec", ctypes.c_int32 * 8),
        ("otype", ctypes.c_int32), ("act", ctypes.c_int32), ("s2", ctypes.c_float), ("eta", ctypes.c_float),
        ("max_batch", ctypes.c_int32), ("device", ctypes.c_int32), ("reserved", ctypes.c_int32 * 4),
    ]


class VaebError(RuntimeError):
    pass


_lib = None

_F = ctypes.POINTER(ctypes.c_float)
_I64 = ctypes.c_int64
_P = ctypes.c_void_p


def load():
    """Load the HIP library (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise VaebError(f"{LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
    if not os.environ.get("VAEB_LIB_VARIANT"):
        from ._buildinfo import check_stamp
        why = check_stamp(LIB_PATH)
        if why:
            raise VaebError(f"stale {LIB_PATH}: {why}; rebuild with `python -c 'import __graft_entry__ as g; g.build()'`")
    lib = ctypes.CDLL(LIB_PATH)
    sig = {
        "vaeb_last_error": ([], ctypes.c_char_p),
        "vaeb_version": ([ctypes.POINTER(ctypes.c_int32)] * 2, ctypes.c_int),
        "vaeb_create": ([ctypes.POINTER(VaebConfig), ctypes.POINTER(_P)], ctypes.c_int),
        "vaeb_destroy": ([_P], ctypes.c_int),
        "vaeb_num_params": ([_P, ctypes.POINTER(_I64)], ctypes.c_int),
        "vaeb_set_data": ([_P, _F, _I64], ctypes.c_int),
        "vaeb_set_params": ([_P, _F, _I64], ctypes.c_int),
        "vaeb_get_params": ([_P, _F, _I64], ctypes.c_int),
        "vaeb_set_adagrad_state": ([_P, _F, _I64], ctypes.c_int),
        "vaeb_get_adagrad_state": ([_P, _F, _I64], ctypes.c_int),
        "vaeb_set_fv_state": ([_P, _F, _F, _F, _F, _I64], ctypes.c_int),
        "vaeb_get_fv_state": ([_P, _F, _F, _F, _F, _I64], ctypes.c_int),
        "vaeb_set_eps_mode": ([_P, ctypes.c_int32, ctypes.c_uint64], ctypes.c_int),
        "vaeb_push_eps": ([_P, _F, _I64, ctypes.c_int32], ctypes.c_int),
        "vaeb_set_step": ([_P, _I64], ctypes.c_int),
        "vaeb_get_step": ([_P, ctypes.POINTER(_I64)], ctypes.c_int),
        "vaeb_comm_count": ([_P, ctypes.POINTER(ctypes.c_int32)], ctypes.c_int),
        "vaeb_set_valid_data": ([_P, _F, _I64], ctypes.c_int),
        "vaeb_validate_resident": ([_P, ctypes.POINTER(ctypes.c_double)], ctypes.c_int),
        "vaeb_checkpoint_save": ([_P, ctypes.c_char_p], ctypes.c_int),
        "vaeb_checkpoint_load": ([_P, ctypes.c_char_p], ctypes.c_int),
        "vaeb_update": ([_P, ctypes.c_int32, _F], ctypes.c_int),
        "vaeb_update_async": ([_P, ctypes.c_int32], ctypes.c_int),
        "vaeb_update_many": ([_P, ctypes.POINTER(ctypes.c_int32), ctypes.c_int32], ctypes.c_int),
        "vaeb_epoch_elbo": ([_P, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_I64)], ctypes.c_int),
        "vaeb_synchronize": ([_P], ctypes.c_int),
        "vaeb_validate": ([_P, _F, _I64, ctypes.POINTER(ctypes.c_double)], ctypes.c_int),
        "vaeb_reconstruct": ([_P, _F, _I64, _F], ctypes.c_int),
        "vaeb_reconstruct_sampled": ([_P, _F, _I64, ctypes.c_int32, _F], ctypes.c_int),
        "vaeb_reconstruct_full": ([_P, _F, _I64, ctypes.c_int32, _F, _F], ctypes.c_int),
        "vaeb_decode": ([_P, _F, _I64, _F, _F], ctypes.c_int),
        "vaeb_comm_unique_id": ([ctypes.POINTER(ctypes.c_uint8)], ctypes.c_int),
        "vaeb_comm_init": ([_P, ctypes.POINTER(ctypes.c_uint8), ctypes.c_int32, ctypes.c_int32], ctypes.c_int),
        "vaeb_get_grads": ([_P, _F, _I64], ctypes.c_int),
        "vaeb_get_activation": ([_P, ctypes.c_char_p, _F, _I64], ctypes.c_int),
        "vaeb_profile_steps": ([_P, ctypes.c_int32, _F, ctypes.POINTER(ctypes.c_int32), ctypes.c_int32,
                                ctypes.POINTER(ctypes.c_int32)], ctypes.c_int),
        "vaeb_kernel_name": ([ctypes.c_int32, ctypes.c_char_p, ctypes.c_int32], ctypes.c_int),
        "vaeb_graph_status": ([_P, ctypes.POINTER(ctypes.c_int32), ctypes.c_char_p, ctypes.c_int32], ctypes.c_int),
        "vaeb_comm_info": ([_P] + [ctypes.POINTER(ctypes.c_int32)] * 3, ctypes.c_int),
        "vaeb_busy": ([_P, ctypes.c_int32], ctypes.c_int),
        "vaeb_dp_plan": ([ctypes.POINTER(VaebConfig)] + [ctypes.c_int32] * 4 +
                         [ctypes.POINTER(_I64), ctypes.POINTER(_I64), ctypes.POINTER(ctypes.c_int32),
                          ctypes.POINTER(_I64), ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32),
                          ctypes.POINTER(_I64), ctypes.POINTER(ctypes.c_int32)], ctypes.c_int),
        "vaeb_dp_rank_update": ([_P] + [ctypes.c_int32] * 3 + [_F, _I64, _F, ctypes.c_int32], ctypes.c_int),
        "vaeb_get_shadow": ([_P, ctypes.POINTER(ctypes.c_uint16), _I64], ctypes.c_int),
        "vaeb_time_update_many": ([_P, ctypes.POINTER(ctypes.c_int32), ctypes.c_int32, _F,
                                   ctypes.POINTER(ctypes.c_double)], ctypes.c_int),
        "vaeb_debug_timeline": ([_P, ctypes.c_int32, ctypes.POINTER(ctypes.c_uint64), _I64,
                                 ctypes.POINTER(ctypes.c_int32)], ctypes.c_int),
        "vaeb_test_gemm_bf16": ([_P] + [ctypes.c_int32] * 5 + [_F, _F, _F, ctypes.c_int32], ctypes.c_int),
        "vaeb_bench_gemm_bf16": ([_P] + [ctypes.c_int32] * 7 + [_F], ctypes.c_int),
        "vaeb_push_fv_noise": ([_P, _F, _I64], ctypes.c_int),
        "vaeb_ae_create": ([ctypes.POINTER(AEConfigC), ctypes.POINTER(_P)], ctypes.c_int),
        "vaeb_ae_destroy": ([_P], ctypes.c_int),
        "vaeb_ae_num_params": ([_P, ctypes.POINTER(_I64)], ctypes.c_int),
        "vaeb_ae_set_data": ([_P, _F, _I64], ctypes.c_int),
        "vaeb_ae_set_params": ([_P, _F, _I64], ctypes.c_int),
        "vaeb_ae_get_params": ([_P, _F, _I64], ctypes.c_int),
        "vaeb_ae_set_adagrad_state": ([_P, _F, _I64], ctypes.c_int),
        "vaeb_ae_get_adagrad_state": ([_P, _F, _I64], ctypes.c_int),
        "vaeb_ae_train": ([_P, ctypes.POINTER(ctypes.c_int32), ctypes.c_int32, _F], ctypes.c_int),
        "vaeb_ae_train_many": ([_P, ctypes.POINTER(ctypes.c_int32), ctypes.c_int32, ctypes.c_int32, _F], ctypes.c_int),
        "vaeb_ae_reconstruct": ([_P, _F, _I64, _F], ctypes.c_int),
        "vaeb_ae_encode": ([_P, _F, _I64, _F], ctypes.c_int),
        "vaeb_ae_decode": ([_P, _F, _I64, _F], ctypes.c_int),
    }
    for name, (args, res) in sig.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res
    _lib = lib
    return lib


def check(rc):
    if rc != 0:
        msg = _lib.vaeb_last_error().decode(errors="replace") if _lib is not None else "?"
        raise VaebError(f"libvaeb_hip error {rc}: {msg}")


def dp_plan(D, H, Z, world, rank, bucket=2, sharded=True, decoder=DEC_BERNOULLI):
    """The sharded DP optimizer's index plan as the library computes it (vaeb_dp_plan; host
    only, no GPU).  bucket 0 = A (W2 | W6), 1 = B, 2 = all.  Returns a dict: P, runs [(lo, n,
    S)], own [(lo, n)], book (bool), foreign [(lo, n)]."""
    lib = load()
    cfg = VaebConfig()
    cfg.D, cfg.H, cfg.Z, cfg.B, cfg.L = D, H, Z, 1, 1
    cfg.decoder = decoder
    P = _I64()
    runs = (_I64 * 9)()
    own = (_I64 * 12)()
    foreign = (_I64 * 12)()
    nrun, nown, book, nfor = (ctypes.c_int32() for _ in range(4))
    check(lib.vaeb_dp_plan(ctypes.byref(cfg), world, rank, int(bool(sharded)), bucket, ctypes.byref(P), runs,
                           ctypes.byref(nrun), own, ctypes.byref(nown), ctypes.byref(book), foreign,
                           ctypes.byref(nfor)))
    return {"P": P.value,
            "runs": [(runs[3 * j], runs[3 * j + 1], runs[3 * j + 2]) for j in range(nrun.value)],
            "own": [(own[2 * k], own[2 * k + 1]) for k in range(nown.value)],
            "book": bool(book.value),
            "foreign": [(foreign[2 * k], foreign[2 * k + 1]) for k in range(nfor.value)]}


def fptr(a: np.ndarray):
    assert a.dtype == np.float32 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(_F)


class Context:
    """Thin RAII wrapper over one vaeb_ctx (one GPU / rank)."""

    def __init__(self, D, H, Z, B, L=1, decoder=DEC_BERNOULLI, estimator=EST_LB, objective=OBJ_SUM_PRIOR,
                 lr=0.01, adagrad_eps=1e-6, device=0, B_global=None, row_offset=0, max_eval_rows=10000,
                 use_graph=True, keep_grads=False, dtype=DTYPE_F32):
        self.lib = load()
        cfg = VaebConfig()
        cfg.D, cfg.H, cfg.Z, cfg.B, cfg.L = D, H, Z, B, L
        cfg.B_global = B if B_global is None else B_global
        cfg.row_offset = row_offset
        cfg.decoder, cfg.estimator, cfg.objective = decoder, estimator, objective
        cfg.lr, cfg.adagrad_eps = lr, adagrad_eps
        cfg.device, cfg.max_eval_rows = device, max_eval_rows
        cfg.use_graph, cfg.keep_grads = int(bool(use_graph)), int(bool(keep_grads))
        cfg.dtype = int(dtype)
        self.cfg = cfg
        self.h = _P()
        check(self.lib.vaeb_create(ctypes.byref(cfg), ctypes.byref(self.h)))
        n = _I64()
        check(self.lib.vaeb_num_params(self.h, ctypes.byref(n)))
        self.P = n.value

    def close(self):
        if getattr(self, "h", None) is not None and self.h.value:
            self.lib.vaeb_destroy(self.h)
            self.h = _P()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- state
    def set_data(self, x):
        x = np.ascontiguousarray(x, np.float32)
        check(self.lib.vaeb_set_data(self.h, fptr(x), x.shape[0]))

    def set_params(self, flat):
        flat = np.ascontiguousarray(flat, np.float32)
        check(self.lib.vaeb_set_params(self.h, fptr(flat), flat.size))

    def get_params(self):
        out = np.empty(self.P, np.float32)
        check(self.lib.vaeb_get_params(self.h, fptr(out), out.size))
        return out

    def set_adagrad_state(self, flat):
        flat = np.ascontiguousarray(flat, np.float32)
        check(self.lib.vaeb_set_adagrad_state(self.h, fptr(flat), flat.size))

    def get_adagrad_state(self):
        out = np.empty(self.P, np.float32)
        check(self.lib.vaeb_get_adagrad_state(self.h, fptr(out), out.size))
        return out

    def get_grads(self):
        out = np.empty(self.P, np.float32)
        check(self.lib.vaeb_get_grads(self.h, fptr(out), out.size))
        return out

    def set_fv_state(self, mu, sigma, acc_mu, acc_sigma):
        arrs = [np.ascontiguousarray(a, np.float32) for a in (mu, sigma, acc_mu, acc_sigma)]
        check(self.lib.vaeb_set_fv_state(self.h, *[fptr(a) for a in arrs], arrs[0].size))

    def get_fv_state(self):
        arrs = [np.empty(self.P, np.float32) for _ in range(4)]
        check(self.lib.vaeb_get_fv_state(self.h, *[fptr(a) for a in arrs], self.P))
        return arrs

    def activation(self, name, n):
        out = np.empty(n, np.float32)
        check(self.lib.vaeb_get_activation(self.h, name.encode(), fptr(out), n))
        return out

    # ---- noise
    def set_eps_mode(self, mode, seed=10):
        check(self.lib.vaeb_set_eps_mode(self.h, mode, seed))

    def push_fv_noise(self, zeta):
        """VAEB_EST_FVS, host eps mode: zeta [P] for the next step's theta~ = mu + |sigma| zeta."""
        zeta = np.ascontiguousarray(zeta, np.float32).ravel()
        check(self.lib.vaeb_push_fv_noise(self.h, fptr(zeta), zeta.size))

    def push_eps(self, eps):
        eps = np.ascontiguousarray(eps, np.float32)
        L, rows, _ = eps.shape
        check(self.lib.vaeb_push_eps(self.h, fptr(eps), rows, L))

    def set_step(self, step):
        check(self.lib.vaeb_set_step(self.h, int(step)))

    def get_step(self):
        n = _I64()
        check(self.lib.vaeb_get_step(self.h, ctypes.byref(n)))
        return n.value

    # ---- native checkpoint (theta, Adagrad state, Philox seed / step, FV state)
    def checkpoint_save(self, path):
        """path None: join a sharded DP gather without writing (every rank calls it at world > 1)."""
        check(self.lib.vaeb_checkpoint_save(self.h, None if path is None else os.fsencode(path)))

    def checkpoint_load(self, path):
        check(self.lib.vaeb_checkpoint_load(self.h, os.fsencode(path)))

    # ---- steps
    def update(self, index):
        out = ctypes.c_float()
        check(self.lib.vaeb_update(self.h, int(index), ctypes.byref(out)))
        return out.value

    def update_async(self, index):
        """One step enqueued without waiting (its value joins the epoch sums)."""
        check(self.lib.vaeb_update_async(self.h, int(index)))

    def update_many(self, indices):
        idx = np.ascontiguousarray(indices, np.int32)
        check(self.lib.vaeb_update_many(self.h, idx.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), idx.size))

    def epoch_elbo(self):
        s = ctypes.c_double()
        n = _I64()
        check(self.lib.vaeb_epoch_elbo(self.h, ctypes.byref(s), ctypes.byref(n)))
        return s.value, n.value

    def synchronize(self):
        check(self.lib.vaeb_synchronize(self.h))

    def validate(self, x):
        x = np.ascontiguousarray(x, np.float32)
        out = ctypes.c_double()
        check(self.lib.vaeb_validate(self.h, fptr(x), x.shape[0], ctypes.byref(out)))
        return out.value

    def set_valid_data(self, x):
        """Upload the validation set once (device-resident, VAEB.py:582's x_valid)."""
        x = np.ascontiguousarray(x, np.float32)
        check(self.lib.vaeb_set_valid_data(self.h, fptr(x), x.shape[0]))

    def validate_resident(self):
        """SGVB sum over the resident validation set (this rank's share, all-reduced)."""
        out = ctypes.c_double()
        check(self.lib.vaeb_validate_resident(self.h, ctypes.byref(out)))
        return out.value

    def reconstruct(self, x):
        x = np.ascontiguousarray(x, np.float32)
        y = np.empty((x.shape[0], self.cfg.D), np.float32)
        check(self.lib.vaeb_reconstruct(self.h, fptr(x), x.shape[0], fptr(y)))
        return y

    def reconstruct_sampled(self, x, n_samples):
        """Decoder output averaged over n_samples posterior draws (VAEB.py:271-291)."""
        x = np.ascontiguousarray(x, np.float32)
        y = np.empty((x.shape[0], self.cfg.D), np.float32)
        check(self.lib.vaeb_reconstruct_sampled(self.h, fptr(x), x.shape[0], int(n_samples), fptr(y)))
        return y

    def reconstruct_full(self, x, n_samples=0, log_sigma=True):
        """(y, y_log_sigma): decoder mean and (Gaussian decoder) log-sigma head, at z = mu or
        averaged over n_samples posterior draws (VAEB.py:267-291); y_log_sigma is None for
        the Bernoulli decoder or when log_sigma is False."""
        x = np.ascontiguousarray(x, np.float32)
        y = np.empty((x.shape[0], self.cfg.D), np.float32)
        lv = np.empty_like(y) if (log_sigma and self.cfg.decoder == DEC_GAUSSIAN) else None
        check(self.lib.vaeb_reconstruct_full(self.h, fptr(x), x.shape[0], int(n_samples), fptr(y),
                                             fptr(lv) if lv is not None else None))
        return y, lv

    def decode(self, z, log_sigma=True):
        """(mu, log_sigma) of the decoder at given latents z [n x Z] (freyFace.py:173-187,
        237-245); log_sigma is None for the Bernoulli decoder or when not requested."""
        z = np.ascontiguousarray(np.atleast_2d(z), np.float32)
        if z.shape[1] != self.cfg.Z:
            raise VaebError(f"decode: z has {z.shape[1]} columns, the model's latent size is {self.cfg.Z}")
        mu = np.empty((z.shape[0], self.cfg.D), np.float32)
        lv = np.empty_like(mu) if (log_sigma and self.cfg.decoder == DEC_GAUSSIAN) else None
        check(self.lib.vaeb_decode(self.h, fptr(z), z.shape[0], fptr(mu), fptr(lv) if lv is not None else None))
        return mu, lv

    def time_update_many(self, indices):
        """(GPU ms, host enqueue ms) of one update_many call (diagnostics)."""
        idx = np.ascontiguousarray(indices, np.int32)
        g, h = ctypes.c_float(), ctypes.c_double()
        check(self.lib.vaeb_time_update_many(self.h, idx.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), idx.size,
                                             ctypes.byref(g), ctypes.byref(h)))
        return g.value, h.value

    def busy(self, us):
        """Diagnostics: every CU busy for `us` microseconds on the context's stream."""
        check(self.lib.vaeb_busy(self.h, int(us)))

    def graph_status(self):
        """(mode, message): 'off' | 'not_captured' | 'replay' | 'eager_fallback' (message: why)."""
        m = ctypes.c_int32()
        buf = ctypes.create_string_buffer(512)
        check(self.lib.vaeb_graph_status(self.h, ctypes.byref(m), buf, 512))
        return GRAPH_MODES[m.value], buf.value.decode(errors="replace")

    def comm_info(self):
        """{'rccl_version', 'dp_overlap' (None without a communicator), 'world'}."""
        v, o, w = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
        check(self.lib.vaeb_comm_info(self.h, ctypes.byref(v), ctypes.byref(o), ctypes.byref(w)))
        return {"rccl_version": v.value, "dp_overlap": None if o.value < 0 else bool(o.value), "world": w.value}

    # ---- data parallel
    @staticmethod
    def comm_unique_id():
        lib = load()
        buf = (ctypes.c_uint8 * 128)()
        check(lib.vaeb_comm_unique_id(buf))
        return bytes(buf)

    def comm_init(self, uid: bytes, rank, world):
        buf = (ctypes.c_uint8 * 128).from_buffer_copy(uid)
        check(self.lib.vaeb_comm_init(self.h, buf, rank, world))

    def comm_count(self):
        """Ranks in the library's RCCL communicator (ncclCommCount); 1 without one."""
        n = ctypes.c_int32()
        check(self.lib.vaeb_comm_count(self.h, ctypes.byref(n)))
        return n.value

    def dp_rank_update(self, world, rank, bucket, grad_sum, theta_gathered=None, finish=False):
        """Diagnostics: rank `rank` of a `world`-rank sharded DP optimizer step for one bucket on
        this (communicator-less) context, the collectives emulated by host copies
        (include/vaeb_diag.h vaeb_dp_rank_update).  grad_sum: [P + 1] summed gradient | SGVB;
        theta_gathered: [P] the other ranks' theta' (the all-gather) or None."""
        g = np.ascontiguousarray(grad_sum, np.float32)
        t = None if theta_gathered is None else np.ascontiguousarray(theta_gathered, np.float32)
        if t is not None and t.size != self.P:
            raise VaebError(f"theta_gathered holds {t.size} floats, expected {self.P}")
        check(self.lib.vaeb_dp_rank_update(self.h, int(world), int(rank), int(bucket), fptr(g), g.size,
                                           fptr(t) if t is not None else None, int(bool(finish))))

    def get_shadow(self, n_weights):
        """Diagnostics (bf16 engine): the bf16 shadow of the weight elements, arena order, as raw
        uint16 bits."""
        out = np.empty(int(n_weights), np.uint16)
        check(self.lib.vaeb_get_shadow(self.h, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint16)), out.size))
        return out

    def bench_gemm_bf16(self, a_kouter, b_kouter, M, N, K, tile_n=0, reps=10):
        """Mean ms per launch of the bf16 GEMM on device-generated operands (diagnostics)."""
        out = ctypes.c_float()
        check(self.lib.vaeb_bench_gemm_bf16(self.h, int(a_kouter), int(b_kouter), M, N, K, int(tile_n), int(reps),
                                            ctypes.byref(out)))
        return out.value

    def test_gemm_bf16(self, A, B, a_kouter, b_kouter, M, N, K, ksplit=1):
        """bf16 GEMM engine test hook: C[M x N] = sum_k A(m,k) B(k,n); A stored [M,K] or
        (a_kouter) [K,M], B stored [N,K] or (b_kouter) [K,N]."""
        A = np.ascontiguousarray(A, np.float32)
        B = np.ascontiguousarray(B, np.float32)
        C = np.empty((M, N), np.float32)
        check(self.lib.vaeb_test_gemm_bf16(self.h, int(a_kouter), int(b_kouter), M, N, K, fptr(A), fptr(B), fptr(C),
                                           int(ksplit)))
        return C

    # ---- measurement
    def debug_timeline(self, batch_index=0):
        """[launch][workgroup][slot] 100 MHz stamps of one eager step (diagnostics)."""
        out = np.zeros(16 * 1024 * 8, np.uint64)
        nl = ctypes.c_int32()
        check(self.lib.vaeb_debug_timeline(self.h, int(batch_index), out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
                                           out.size, ctypes.byref(nl)))
        return out.reshape(16, 1024, 8)[:nl.value]

    def profile_steps(self, n_steps):
        ms = np.zeros(32, np.float32)
        ids = np.zeros(32, np.int32)
        nk = ctypes.c_int32()
        check(self.lib.vaeb_profile_steps(self.h, n_steps, fptr(ms), ids.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                          32, ctypes.byref(nk)))
        out = []
        for k in range(nk.value):
            buf = ctypes.create_string_buffer(64)
            check(self.lib.vaeb_kernel_name(int(ids[k]), buf, 64))
            out.append((buf.value.decode(), float(ms[k])))
        return out


class AEContext:
    """One degenerate-vae autoencoder (vaeb_ae_*) on one GPU."""

    def __init__(self, Dobs, Denc, Dz, Ddec, otype="binary", act="tanh", s2=1.0, eta=0.01, max_batch=100,
                 device=0):
        self.lib = load()
        c = AEConfigC()
        c.Dobs, c.Dz = int(Dobs), int(Dz)
        Denc, Ddec = list(Denc), list(Ddec)
        if not (1 <= len(Denc) <= AE_MAX_LAYERS and 1 <= len(Ddec) <= AE_MAX_LAYERS):
            raise VaebError(f"1..{AE_MAX_LAYERS} encoder / decoder hidden layers are supported")
        c.n_enc, c.n_dec = len(Denc), len(Ddec)
        for i, d in enumerate(Denc):
            c.Denc[i] = int(d)
        for i, d in enumerate(Ddec):
            c.Ddec[i] = int(d)
        c.otype = {"binary": AE_BINARY, "cont": AE_CONT}[otype]
        c.act = ACT[act]
        c.s2, c.eta = float(s2), float(eta)
        c.max_batch, c.device = int(max_batch), int(device)
        self.cfg = c
        self.Dobs, self.Dz = c.Dobs, c.Dz
        self.h = _P()
        check(self.lib.vaeb_ae_create(ctypes.byref(c), ctypes.byref(self.h)))
        n = _I64()
        check(self.lib.vaeb_ae_num_params(self.h, ctypes.byref(n)))
        self.P = n.value

    def close(self):
        if getattr(self, "h", None) is not None and self.h.value:
            self.lib.vaeb_ae_destroy(self.h)
            self.h = _P()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_data(self, x):
        x = np.ascontiguousarray(x, np.float32)
        check(self.lib.vaeb_ae_set_data(self.h, fptr(x), x.shape[0]))

    def set_params(self, flat):
        flat = np.ascontiguousarray(flat, np.float32)
        check(self.lib.vaeb_ae_set_params(self.h, fptr(flat), flat.size))

    def get_params(self):
        out = np.empty(self.P, np.float32)
        check(self.lib.vaeb_ae_get_params(self.h, fptr(out), out.size))
        return out

    def set_adagrad_state(self, flat):
        flat = np.ascontiguousarray(flat, np.float32)
        check(self.lib.vaeb_ae_set_adagrad_state(self.h, fptr(flat), flat.size))

    def get_adagrad_state(self):
        out = np.empty(self.P, np.float32)
        check(self.lib.vaeb_ae_get_adagrad_state(self.h, fptr(out), out.size))
        return out

    def train(self, idx):
        idx = np.ascontiguousarray(idx, np.int32)
        out = ctypes.c_float()
        check(self.lib.vaeb_ae_train(self.h, idx.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), idx.size,
                                     ctypes.byref(out)))
        return out.value

    def train_many(self, idx, batch):
        idx = np.ascontiguousarray(idx, np.int32)
        nb = -(-idx.size // int(batch))
        out = np.empty(nb, np.float32)
        check(self.lib.vaeb_ae_train_many(self.h, idx.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), idx.size,
                                          int(batch), fptr(out)))
        return out

    def _predict(self, fn, x, width_out):
        x = np.ascontiguousarray(x, np.float32)
        out = np.empty((x.shape[0], width_out), np.float32)
        check(fn(self.h, fptr(x), x.shape[0], fptr(out)))
        return out

    def reconstruct(self, x):
        return self._predict(self.lib.vaeb_ae_reconstruct, x, self.Dobs)

    def encode(self, x):
        return self._predict(self.lib.vaeb_ae_encode, x, self.Dz)

    def decode(self, z):
        return self._predict(self.lib.vaeb_ae_decode, z, self.Dobs)
