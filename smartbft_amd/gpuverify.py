"""ctypes binding of libsbft_gpuverify.so (include/sbft_gpuverify.h).

This is the product path used by tests and bench.py: every call goes through the C ABI
into the HIP kernels. There is no CPU fallback: if the shared library is missing or no
GPU is visible, construction raises (GpuVerifyError), loudly.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SBFT_GV_LIB") or os.path.join(_HERE, "libsbft_gpuverify.so")

EXPORTS = [
    "sbft_gv_init", "sbft_gv_destroy", "sbft_gv_device_count", "sbft_gv_strerror",
    "sbft_gv_verify_p256", "sbft_gv_sha256", "sbft_gv_sha256_verify_p256",
    "sbft_gv_verify_p256_dev", "sbft_gv_sha256_dev", "sbft_gv_sha256_verify_p256_dev",
    "sbft_gv_normalize_hash", "sbft_gv_normalize_scalar", "sbft_gv_sign_p256", "sbft_gv_sign_p256_dev",
    "sbft_gv_selftest_field", "sbft_gv_verify_workspace_bytes",
    "sbft_gv_register_key", "sbft_gv_verify_p256_keyed", "sbft_gv_sha256_verify_p256_keyed",
    "sbft_gv_kernel_timing", "sbft_gv_kernel_time", "sbft_gv_register_keys",
    "sbft_gv_sha256_verify_p256_framed", "sbft_gv_host_alloc", "sbft_gv_host_free",
    "sbft_gv_plan_split", "sbft_gv_sha256_verify_p256_stream", "sbft_gv_inject_fault",
    "sbft_gv_register_client_keys", "sbft_gv_verify_p256_kernel",
]

_u8p = ctypes.POINTER(ctypes.c_uint8)
_vp = ctypes.c_void_p

# sbft_gv_verify_p256_kernel's kernel names (include/sbft_gpuverify.h)
KERNEL_EXACT, KERNEL_THROUGHPUT, KERNEL_PAIR, KERNEL_HALF, KERNEL_HALF_WIDE = 0, 1, 2, 3, 4


class GpuVerifyError(RuntimeError):
    pass


class Opts(ctypes.Structure):
    _fields_ = [("device_mask", ctypes.c_uint32), ("min_split", ctypes.c_uint32),
                ("pair_max", ctypes.c_int32), ("reserved0", ctypes.c_int32),
                ("slots_per_device", ctypes.c_uint32), ("half_max", ctypes.c_int32),
                ("client_table_bytes", ctypes.c_uint64), ("halfq_max", ctypes.c_int32),
                ("reserved1", ctypes.c_int32)]


_LIB = None


def load_library():
    """Load the HIP shared library (raises if it was not built)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise GpuVerifyError(f"{LIB_PATH} missing: run `make -C smartbft_amd/csrc` "
                             "(or __graft_entry__.build()); there is no CPU fallback")
    L = ctypes.CDLL(LIB_PATH)
    L.sbft_gv_init.argtypes = [ctypes.POINTER(Opts), ctypes.POINTER(_vp)]
    L.sbft_gv_destroy.argtypes = [_vp]
    L.sbft_gv_destroy.restype = None
    L.sbft_gv_device_count.argtypes = [_vp]
    L.sbft_gv_strerror.argtypes = [ctypes.c_int]
    L.sbft_gv_strerror.restype = ctypes.c_char_p
    L.sbft_gv_verify_p256.argtypes = [_vp] + [_u8p] * 5 + [ctypes.c_size_t, _u8p]
    L.sbft_gv_verify_p256_kernel.argtypes = [_vp, ctypes.c_int] + [_u8p] * 5 + [ctypes.c_size_t, _u8p]
    L.sbft_gv_sha256.argtypes = [_vp, _u8p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_uint64),
                                 ctypes.POINTER(ctypes.c_uint32), ctypes.c_size_t, _u8p]
    L.sbft_gv_sha256_verify_p256.argtypes = [_vp, _u8p, ctypes.c_size_t,
                                             ctypes.POINTER(ctypes.c_uint64),
                                             ctypes.POINTER(ctypes.c_uint32)] + [_u8p] * 4 + \
                                            [ctypes.c_size_t, _u8p, _u8p]
    L.sbft_gv_sha256_verify_p256_framed.argtypes = [_vp, _u8p, ctypes.c_size_t,
                                                    ctypes.POINTER(ctypes.c_uint64),
                                                    ctypes.POINTER(ctypes.c_uint32), ctypes.c_size_t,
                                                    ctypes.c_int32, ctypes.c_int32, _u8p]
    L.sbft_gv_verify_p256_dev.argtypes = [_vp, ctypes.c_int] + [_vp] * 5 + [ctypes.c_size_t, _vp, _vp]
    L.sbft_gv_sha256_dev.argtypes = [_vp, ctypes.c_int] + [_vp] * 4 + [ctypes.c_size_t, _vp, _vp]
    L.sbft_gv_sha256_verify_p256_dev.argtypes = [_vp, ctypes.c_int] + [_vp] * 8 + \
                                                [ctypes.c_size_t, _vp, _vp, _vp]
    L.sbft_gv_sign_p256.argtypes = [_vp] + [_u8p] * 3 + [ctypes.c_size_t] + [_u8p] * 5
    L.sbft_gv_sign_p256_dev.argtypes = [_vp, ctypes.c_int] + [_vp] * 3 + [ctypes.c_size_t] + [_vp] * 6
    L.sbft_gv_verify_workspace_bytes.argtypes = [ctypes.c_size_t]
    L.sbft_gv_verify_workspace_bytes.restype = ctypes.c_size_t
    L.sbft_gv_selftest_field.argtypes = [_vp, ctypes.c_int, _u8p, _u8p, ctypes.c_size_t, _u8p]
    L.sbft_gv_inject_fault.argtypes = [ctypes.c_int, ctypes.c_int]
    L.sbft_gv_kernel_timing.argtypes = [_vp, ctypes.c_int]
    L.sbft_gv_kernel_time.argtypes = [_vp, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_double)]
    L.sbft_gv_normalize_hash.argtypes = [_u8p, ctypes.c_size_t, _u8p]
    L.sbft_gv_normalize_hash.restype = None
    L.sbft_gv_normalize_scalar.argtypes = [_u8p, ctypes.c_size_t, _u8p]
    _u32p = ctypes.POINTER(ctypes.c_uint32)
    L.sbft_gv_register_key.argtypes = [_vp, _u8p, _u8p, _u32p]
    L.sbft_gv_register_keys.argtypes = [_vp, _u8p, _u8p, ctypes.c_size_t, _u32p]
    L.sbft_gv_register_client_keys.argtypes = [_vp, _u8p, _u8p, ctypes.c_size_t, _u32p,
                                               ctypes.POINTER(ctypes.c_size_t)]
    L.sbft_gv_verify_p256_keyed.argtypes = [_vp] + [_u8p] * 3 + [_u32p, ctypes.c_size_t, _u8p]
    L.sbft_gv_sha256_verify_p256_keyed.argtypes = [_vp, _u8p, ctypes.c_size_t,
                                                   ctypes.POINTER(ctypes.c_uint64), _u32p, _u8p, _u8p,
                                                   _u32p, ctypes.c_size_t, _u8p]
    L.sbft_gv_host_alloc.argtypes = [ctypes.c_size_t, ctypes.POINTER(_vp)]
    L.sbft_gv_host_free.argtypes = [_vp]
    L.sbft_gv_host_free.restype = None
    L.sbft_gv_sha256_verify_p256_stream.argtypes = [_vp, _u8p, ctypes.c_size_t,
                                                    ctypes.POINTER(ctypes.c_uint64),
                                                    ctypes.POINTER(ctypes.c_uint32)] + [_u8p] * 4 + \
                                                   [ctypes.c_size_t, ctypes.c_size_t, _u8p, _u8p]
    _szp = ctypes.POINTER(ctypes.c_size_t)
    L.sbft_gv_plan_split.argtypes = [ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t, _szp, _szp]
    L.sbft_gv_plan_split.restype = ctypes.c_size_t
    _LIB = L
    return L


class PinnedArray:
    """Page-locked host memory from sbft_gv_host_alloc, seen as a uint8 numpy array of the
    given shape. Verify inputs held in these let sbft_gv_verify_p256 overlap its H2D copies
    with the kernels. Free with close() (the numpy view must not be used afterwards)."""

    def __init__(self, shape):
        self.L = load_library()
        n = int(np.prod(shape))
        ptr = _vp()
        rc = self.L.sbft_gv_host_alloc(n, ctypes.byref(ptr))
        if rc:
            raise GpuVerifyError(f"sbft_gv_host_alloc: {self.L.sbft_gv_strerror(rc).decode()} ({rc})")
        self.ptr = ptr
        buf = (ctypes.c_uint8 * max(n, 1)).from_address(ptr.value) if n else bytearray(1)
        self.array = np.frombuffer(buf, dtype=np.uint8, count=n).reshape(shape)

    def close(self):
        if getattr(self, "ptr", None):
            self.array = None
            self.L.sbft_gv_host_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _p(a: np.ndarray):
    return a.ctypes.data_as(_u8p)


def _soa(a, n: int) -> np.ndarray:
    a = np.ascontiguousarray(np.asarray(a, dtype=np.uint8))
    if a.shape != (n, 32):
        raise ValueError(f"expected ({n}, 32) uint8, got {a.shape}")
    return a


def _msgs(blob, off, ln):
    """Host-side message batch: contiguous uint8 blob, uint64 offsets and uint32 lengths of
    one length n each (the C side reads len[k] / off[k] for every k < n)."""
    blob = np.ascontiguousarray(blob, dtype=np.uint8).reshape(-1)
    off = np.ascontiguousarray(off, dtype=np.uint64).reshape(-1)
    ln = np.ascontiguousarray(ln, dtype=np.uint32).reshape(-1)
    if ln.shape != off.shape:
        raise ValueError(f"offsets {off.shape} and lengths {ln.shape} differ")
    return blob, off, ln, off.shape[0]


def _key_ids(key_ids, n: int) -> np.ndarray:
    kid = np.ascontiguousarray(key_ids, dtype=np.uint32).reshape(-1)
    if kid.shape != (n,):
        raise ValueError(f"expected {n} key ids, got {kid.shape}")
    return kid


def _dev(t, numel: int, what: str, dtype=None):
    """A device tensor the C side reads or writes numel elements of, densely."""
    import torch
    if not t.is_cuda:
        raise ValueError(f"{what}: expected a HIP device tensor")
    if not t.is_contiguous():
        raise ValueError(f"{what}: tensor must be contiguous")
    if t.numel() != numel:
        raise ValueError(f"{what}: expected {numel} elements, got {t.numel()}")
    if t.dtype != (dtype or torch.uint8):
        raise ValueError(f"{what}: expected {dtype or torch.uint8}, got {t.dtype}")
    return t.data_ptr()


def plan_split(n: int, n_devices: int, min_split: int = 0) -> list[tuple[int, int]]:
    """The library's host-side batch split (sbft_gv_plan_split, no GPU): [(begin, count)], one
    contiguous share per device."""
    L = load_library()
    b = (ctypes.c_size_t * max(1, n_devices))()
    c = (ctypes.c_size_t * max(1, n_devices))()
    m = L.sbft_gv_plan_split(n, n_devices, min_split, b, c)
    return [(b[i], c[i]) for i in range(m)]


def normalize_hash(h: bytes) -> bytes:
    L = load_library()
    out = (ctypes.c_uint8 * 32)()
    buf = (ctypes.c_uint8 * max(1, len(h))).from_buffer_copy(h or b"\0")
    L.sbft_gv_normalize_hash(buf, len(h), out)
    return bytes(out)


def normalize_scalar(be: bytes) -> bytes | None:
    L = load_library()
    out = (ctypes.c_uint8 * 32)()
    buf = (ctypes.c_uint8 * max(1, len(be))).from_buffer_copy(be or b"\0")
    return bytes(out) if L.sbft_gv_normalize_scalar(buf, len(be), out) else None


FAULT_OFF, FAULT_NOMEM, FAULT_LAUNCH, FAULT_SYNC = 0, 1, 2, 3


def inject_fault(kind: int, count: int = -1) -> None:
    """Arm a process-wide engine fault (sbft_gv_inject_fault; tests of the error paths): the next
    `count` fault points of `kind` fail (-1: every one until inject_fault(FAULT_OFF))."""
    rc = load_library().sbft_gv_inject_fault(kind, count)
    if rc:
        raise GpuVerifyError(f"sbft_gv_inject_fault: {rc}")


class GpuVerifier:
    """One sbft_gv_ctx. Host-array calls are synchronous; *_dev calls take torch tensors
    (device-resident) and enqueue on the given (or current) stream."""

    def __init__(self, device_mask: int = 0, min_split: int = 0, pair_max: int = 0,
                 slots_per_device: int = 0, half_max: int = 0, client_table_bytes: int = 0,
                 halfq_max: int = 0):
        """pair_max / half_max / halfq_max: per-device batches of at most this many tuples run the
        pair latency kernel (two lanes per tuple) / the half-size-scalar kernel (four lanes: two
        128-bit ladders) / its wide form (eight lanes: a quad per ladder), halfq_max then half_max
        taking precedence (0 = library default, negative = never; pair_max < 0 with half_max 0
        forces the one-lane throughput kernel).
        slots_per_device > 1: that many engine slots per GPU, each taking a share of a split
        batch as a separate device would (runs the multi-device split on one GPU).
        client_table_bytes: per-device budget of client-key comb tables (0 = 1/8 of the device)."""
        self.L = load_library()
        ctx = _vp()
        opts = Opts(device_mask, min_split, pair_max, 0, slots_per_device, half_max, client_table_bytes,
                    halfq_max, 0)
        rc = self.L.sbft_gv_init(ctypes.byref(opts), ctypes.byref(ctx))
        if rc:
            raise GpuVerifyError(f"sbft_gv_init: {self.L.sbft_gv_strerror(rc).decode()} ({rc})")
        self.ctx = ctx

    def close(self):
        if getattr(self, "ctx", None):
            self.L.sbft_gv_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc, what):
        if rc:
            raise GpuVerifyError(f"{what}: {self.L.sbft_gv_strerror(rc).decode()} ({rc})")

    @property
    def device_count(self) -> int:
        return self.L.sbft_gv_device_count(self.ctx)

    def verify(self, digest, r, s, qx, qy) -> np.ndarray:
        n = len(digest)
        arrs = [_soa(a, n) for a in (digest, r, s, qx, qy)]
        ok = np.zeros(n, dtype=np.uint8)
        self._check(self.L.sbft_gv_verify_p256(self.ctx, *[_p(a) for a in arrs], n, _p(ok)),
                    "sbft_gv_verify_p256")
        return ok

    def verify_kernel(self, kernel: int, digest, r, s, qx, qy) -> np.ndarray:
        """sbft_gv_verify_p256_kernel: the same verify on a named kernel (KERNEL_EXACT,
        KERNEL_THROUGHPUT, KERNEL_PAIR, KERNEL_HALF, KERNEL_HALF_WIDE)."""
        n = len(digest)
        arrs = [_soa(a, n) for a in (digest, r, s, qx, qy)]
        ok = np.zeros(n, dtype=np.uint8)
        self._check(self.L.sbft_gv_verify_p256_kernel(self.ctx, kernel, *[_p(a) for a in arrs], n, _p(ok)),
                    "sbft_gv_verify_p256_kernel")
        return ok

    def register_key(self, qx: bytes, qy: bytes) -> int:
        """Precompute the comb tables of a (consenter) key; returns its key id (>= 1). Raises
        GpuVerifyError for a key that is not a valid P-256 point."""
        kx = (ctypes.c_uint8 * 32).from_buffer_copy(bytes(qx))
        ky = (ctypes.c_uint8 * 32).from_buffer_copy(bytes(qy))
        kid = ctypes.c_uint32()
        self._check(self.L.sbft_gv_register_key(self.ctx, kx, ky, ctypes.byref(kid)), "sbft_gv_register_key")
        return kid.value

    def register_keys(self, qx, qy, client: bool = False) -> np.ndarray:
        """Batch registration (one table-build launch per device): key ids, 0 for invalid keys.
        client=True: sbft_gv_register_client_keys, under the client-table budget (keys past it
        also get id 0)."""
        n = len(qx)
        if n and isinstance(qx[0], (bytes, bytearray)):
            qx = np.frombuffer(b"".join(qx), dtype=np.uint8).reshape(n, 32)
            qy = np.frombuffer(b"".join(qy), dtype=np.uint8).reshape(n, 32)
        ax, ay = _soa(qx, n), _soa(qy, n)
        ids = np.zeros(n, dtype=np.uint32)
        pids = ids.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))
        if client:
            got = ctypes.c_size_t()
            self._check(self.L.sbft_gv_register_client_keys(self.ctx, _p(ax), _p(ay), n, pids, ctypes.byref(got)),
                        "sbft_gv_register_client_keys")
            assert got.value == int(np.count_nonzero(ids))
        else:
            self._check(self.L.sbft_gv_register_keys(self.ctx, _p(ax), _p(ay), n, pids), "sbft_gv_register_keys")
        return ids

    def verify_keyed(self, digest, r, s, key_ids) -> np.ndarray:
        n = len(digest)
        arrs = [_soa(a, n) for a in (digest, r, s)]
        kid = _key_ids(key_ids, n)
        ok = np.zeros(n, dtype=np.uint8)
        self._check(self.L.sbft_gv_verify_p256_keyed(
            self.ctx, *[_p(a) for a in arrs], kid.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), n, _p(ok)),
            "sbft_gv_verify_p256_keyed")
        return ok

    def sha256_verify_keyed(self, blob, off, ln, r, s, key_ids) -> np.ndarray:
        blob, off, ln, n = _msgs(blob, off, ln)
        arrs = [_soa(a, n) for a in (r, s)]
        kid = _key_ids(key_ids, n)
        ok = np.zeros(n, dtype=np.uint8)
        self._check(self.L.sbft_gv_sha256_verify_p256_keyed(
            self.ctx, _p(blob) if blob.size else None, blob.size,
            off.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), ln.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)),
            *[_p(a) for a in arrs], kid.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), n, _p(ok)),
            "sbft_gv_sha256_verify_p256_keyed")
        return ok

    def sign(self, d, k, digest):
        """Q = d*G and ECDSA (r, s) with nonces k. Returns (qx, qy, r, s, status)."""
        n = len(d)
        ins = [_soa(a, n) for a in (d, k, digest)]
        outs = [np.zeros((n, 32), dtype=np.uint8) for _ in range(4)]
        st = np.zeros(n, dtype=np.uint8)
        self._check(self.L.sbft_gv_sign_p256(self.ctx, *[_p(a) for a in ins], n,
                                             *[_p(a) for a in outs], _p(st)), "sbft_gv_sign_p256")
        return (*outs, st)

    def selftest_field(self, op: int, a, b) -> np.ndarray:
        n = len(a)
        a, b = _soa(a, n), _soa(b, n)
        out = np.zeros((n, 32), dtype=np.uint8)
        self._check(self.L.sbft_gv_selftest_field(self.ctx, op, _p(a), _p(b), n, _p(out)),
                    "sbft_gv_selftest_field")
        return out

    def sign_dev(self, d_d, d_k, d_e, d_qx, d_qy, d_r, d_s, d_status, stream=None):
        n = d_status.numel()
        p = [_dev(t, 32 * n, w) for t, w in ((d_d, "d"), (d_k, "k"), (d_e, "digest"), (d_qx, "qx"),
                                             (d_qy, "qy"), (d_r, "r"), (d_s, "s"))]
        self._check(self.L.sbft_gv_sign_p256_dev(
            self.ctx, d_status.device.index, p[0], p[1], p[2], n, p[3], p[4], p[5], p[6],
            _dev(d_status, n, "status"), self._stream(stream, d_status.device)), "sbft_gv_sign_p256_dev")

    def sha256(self, blob: np.ndarray, off: np.ndarray, ln: np.ndarray) -> np.ndarray:
        blob, off, ln, n = _msgs(blob, off, ln)
        dig = np.zeros((n, 32), dtype=np.uint8)
        self._check(self.L.sbft_gv_sha256(self.ctx, _p(blob) if blob.size else None, blob.size,
                                          off.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
                                          ln.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), n,
                                          _p(dig)), "sbft_gv_sha256")
        return dig

    def sha256_verify(self, blob, off, ln, r, s, qx, qy, want_digests=False):
        blob, off, ln, n = _msgs(blob, off, ln)
        arrs = [_soa(a, n) for a in (r, s, qx, qy)]
        ok = np.zeros(n, dtype=np.uint8)
        dig = np.zeros((n, 32), dtype=np.uint8) if want_digests else None
        self._check(self.L.sbft_gv_sha256_verify_p256(
            self.ctx, _p(blob) if blob.size else None, blob.size,
            off.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
            ln.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), *[_p(a) for a in arrs], n, _p(ok),
            _p(dig) if dig is not None else None), "sbft_gv_sha256_verify_p256")
        return (ok, dig) if want_digests else ok

    def sha256_verify_stream(self, blob, off, ln, r, s, qx, qy, window_bytes: int = 0, want_digests=False):
        """Streamed hash + verify (sbft_gv_sha256_verify_p256_stream): windows of about
        window_bytes of payload through double-buffered pinned staging, one host thread per
        device. blob may be a PinnedArray's array (then dense windows are DMA'd in place)."""
        if not (isinstance(blob, np.ndarray) and blob.dtype == np.uint8 and blob.flags.c_contiguous):
            blob = np.ascontiguousarray(blob, dtype=np.uint8)
        blob = blob.reshape(-1)
        _, off, ln, n = _msgs(blob[:0], off, ln)
        arrs = [_soa(a, n) for a in (r, s, qx, qy)]
        ok = np.zeros(n, dtype=np.uint8)
        dig = np.zeros((n, 32), dtype=np.uint8) if want_digests else None
        self._check(self.L.sbft_gv_sha256_verify_p256_stream(
            self.ctx, _p(blob) if blob.size else None, blob.size,
            off.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
            ln.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), *[_p(a) for a in arrs], n, window_bytes,
            _p(ok), _p(dig) if dig is not None else None), "sbft_gv_sha256_verify_p256_stream")
        return (ok, dig) if want_digests else ok

    def sha256_verify_framed(self, blob, off, ln, sig_rel: int, pub_rel: int) -> np.ndarray:
        """Hash + verify of messages whose r || s and x || y sit in the blob at message end
        + sig_rel / + pub_rel (sbft_gv_sha256_verify_p256_framed)."""
        blob, off, ln, n = _msgs(blob, off, ln)
        ok = np.zeros(n, dtype=np.uint8)
        self._check(self.L.sbft_gv_sha256_verify_p256_framed(
            self.ctx, _p(blob) if blob.size else None, blob.size,
            off.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
            ln.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), n, sig_rel, pub_rel, _p(ok)),
            "sbft_gv_sha256_verify_p256_framed")
        return ok

    # ---- device-resident (torch tensors on a HIP device) ----
    @staticmethod
    def _stream(stream, device=None):
        """The given stream, else the current stream of `device` (the device the call's
        tensors live on: a stream of another device would be invalid for the launch)."""
        import torch
        s = stream if stream is not None else torch.cuda.current_stream(device)
        return ctypes.c_void_p(s.cuda_stream)

    @staticmethod
    def _check_blob_bounds(d_blob, d_off, d_len, stream, device):
        """Every message [off, off + len) inside the blob. The reduction runs on the launch stream
        (so offsets still being written there are read after their producer) and its result is
        read back, which synchronises that stream: callers that need the launch to stay
        asynchronous validate their offsets themselves and pass check=False. uint64 offsets at
        or above 2^63 are rejected, not wrapped."""
        import torch
        s = stream if stream is not None else torch.cuda.current_stream(device)
        with torch.cuda.stream(s):
            if bool(GpuVerifier._blob_bounds_bad(d_off, d_len, d_blob.numel()).any()):
                raise ValueError("a message extends past the end of the blob (or its offset is >= 2^63)")

    @staticmethod
    def _blob_bounds_bad(d_off, d_len, blob_bytes: int):
        """Per message: True unless [off, off + len) lies inside a blob of blob_bytes bytes (any
        device; tests/test_abi.py runs it on CPU tensors). off + len is never formed: it wraps
        for an offset near 2^63 (a uint64 offset >= 2^63 reads as negative int64)."""
        import torch
        off = d_off.view(torch.int64) if d_off.dtype == torch.uint64 else d_off.to(torch.int64)
        ln = d_len.view(torch.int32).to(torch.int64) & 0xFFFFFFFF
        return (off < 0) | (ln > blob_bytes) | (off > blob_bytes - ln)

    def verify_dev(self, d_digest, d_r, d_s, d_qx, d_qy, d_ok, stream=None):
        n = d_ok.numel()
        dev = d_ok.device.index
        p = [_dev(t, 32 * n, w) for t, w in ((d_digest, "digest"), (d_r, "r"), (d_s, "s"), (d_qx, "qx"),
                                             (d_qy, "qy"))]
        self._check(self.L.sbft_gv_verify_p256_dev(
            self.ctx, dev, *p, n, _dev(d_ok, n, "ok"), self._stream(stream, d_ok.device)), "sbft_gv_verify_p256_dev")

    def sha256_verify_dev(self, d_blob, d_off, d_len, d_r, d_s, d_qx, d_qy, d_ok, d_dig, stream=None,
                          check: bool = True):
        """Device-resident hash + verify (sbft_gv_sha256_verify_p256_dev): digests of the
        messages land in d_dig and feed the verify of the same tuples on the same stream.
        check=True validates the offsets against the blob first (_check_blob_bounds: this
        synchronises the launch stream)."""
        import torch
        n = d_ok.numel()
        if d_off.dtype not in (torch.int64, torch.uint64) or d_len.dtype not in (torch.int32, torch.uint32):
            raise ValueError("offsets must be 64-bit and lengths 32-bit integers")
        if d_blob.dtype != torch.uint8 or not d_blob.is_contiguous() or not d_blob.is_cuda:
            raise ValueError("blob: expected a contiguous uint8 device tensor")
        if n and check:
            self._check_blob_bounds(d_blob, d_off, d_len, stream, d_ok.device)
        p = [_dev(t, 32 * n, w) for t, w in ((d_r, "r"), (d_s, "s"), (d_qx, "qx"), (d_qy, "qy"))]
        self._check(self.L.sbft_gv_sha256_verify_p256_dev(
            self.ctx, d_ok.device.index, d_blob.data_ptr(), _dev(d_off, n, "offsets", d_off.dtype),
            _dev(d_len, n, "lengths", d_len.dtype), None, *p, n, _dev(d_ok, n, "ok"),
            _dev(d_dig, 32 * n, "digests"), self._stream(stream, d_ok.device)), "sbft_gv_sha256_verify_p256_dev")

    def kernel_timing(self, enable: bool):
        """Record HIP events around each device-resident verify's main kernel."""
        self._check(self.L.sbft_gv_kernel_timing(self.ctx, int(enable)), "sbft_gv_kernel_timing")

    def kernel_time(self) -> tuple[int, float]:
        """(timed launches, summed milliseconds) since the last read."""
        n, ms = ctypes.c_uint64(), ctypes.c_double()
        self._check(self.L.sbft_gv_kernel_time(self.ctx, ctypes.byref(n), ctypes.byref(ms)), "sbft_gv_kernel_time")
        return n.value, ms.value

    def sha256_dev(self, d_blob, d_off, d_len, d_dig, stream=None, d_order=None, check: bool = True):
        """d_off int64/uint64 offsets, d_len int32 lengths, d_order (optional) int32 permutation;
        the hash kernel reads nothing outside the 16-byte granules holding message bytes, so
        the blob needs no padding; check=True validates offsets + lengths against its size on the
        launch stream first (_check_blob_bounds: this synchronises that stream)."""
        import torch
        n = d_off.numel()
        if d_blob.dtype != torch.uint8 or not d_blob.is_contiguous() or not d_blob.is_cuda:
            raise ValueError("blob: expected a contiguous uint8 device tensor")
        if d_off.dtype not in (torch.int64, torch.uint64):
            raise ValueError(f"offsets: expected 64-bit integers, got {d_off.dtype}")
        p_off = _dev(d_off, n, "offsets", d_off.dtype)
        if d_len.dtype not in (torch.int32, torch.uint32):
            raise ValueError(f"lengths: expected 32-bit integers, got {d_len.dtype}")
        if n and check:
            self._check_blob_bounds(d_blob, d_off, d_len, stream, d_dig.device)
        p_len = _dev(d_len, n, "lengths", d_len.dtype)
        p_ord = _dev(d_order, n, "order", d_order.dtype if d_order.dtype in (torch.int32, torch.uint32)
                     else torch.int32) if d_order is not None else None
        self._check(self.L.sbft_gv_sha256_dev(self.ctx, d_dig.device.index, d_blob.data_ptr(), p_off, p_len,
                                              p_ord, n, _dev(d_dig, 32 * n, "digests"), self._stream(stream, d_dig.device)),
                    "sbft_gv_sha256_dev")
