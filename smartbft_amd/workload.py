"""Synthetic signed workloads of BASELINE.json config 2 ("1M ECDSA P-256 verifies, 32-byte
SHA-256 digests, 10% corrupted sigs"), generated on the GPU by the engine itself (its
SHA-256 and signer kernels) so that bench setup takes seconds, not CPU-minutes.

Tuple i (global index; rank r of a multi-GPU run owns [r*N, (r+1)*N)):
  d_i = SHA-256(seed | "key" | le64(i)) mod n      (distinct key per tuple)
  m_i = SHA-256(seed | "msg" | le64(i)) || SHA-256(seed | "ms2" | le64(i))   (64-byte message)
  e_i = SHA-256(m_i)                                (the 32-byte digest that is verified)
  k_i = SHA-256(seed | "k" | le64(i)) mod n         (nonce)
  corrupted iff SHA-256(seed | "c" | le64(i))[0] < 26   (~10.2%)
  corruption kind = (i mod 7): flip an r bit, flip an s bit, flip an e bit, r = 0,
  s = n, Q off-curve (y xor 1), Q replaced by the neighbour's key.
seed = b"SBFT-GPUV-1".
"""
from __future__ import annotations

import numpy as np
import torch

SEED = b"SBFT-GPUV-1"
N_BYTES = bytes.fromhex("FFFFFFFF00000000FFFFFFFFFFFFFFFFBCE6FAADA7179E84F3B9CAC2FC632551")


def _tag_messages(tag: bytes, start: int, n: int) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
    """Fixed-width messages seed|tag|le64(i) for i in [start, start+n) as (blob, off, len)."""
    head = np.frombuffer(SEED + tag, dtype=np.uint8)
    w = len(head) + 8
    blob = np.empty((n, w), dtype=np.uint8)
    blob[:, :len(head)] = head
    idx = np.arange(start, start + n, dtype=np.uint64)
    blob[:, len(head):] = idx.view(np.uint8).reshape(n, 8)
    off = (np.arange(n, dtype=np.uint64) * w)
    ln = np.full(n, w, dtype=np.uint32)
    return blob.reshape(-1), off, ln


def _gpu_sha(gv, blob: np.ndarray, off: np.ndarray, ln: np.ndarray, dev) -> torch.Tensor:
    pad = np.zeros(blob.size + 256, dtype=np.uint8)  # SBFT_GV_SHA_BLOB_PAD
    pad[:blob.size] = blob
    d_blob = torch.from_numpy(pad).to(dev)
    d_off = torch.from_numpy(off.astype(np.int64)).to(dev)
    d_len = torch.from_numpy(ln.astype(np.int32)).to(dev)
    d_dig = torch.empty((len(off), 32), dtype=torch.uint8, device=dev)
    gv.sha256_dev(d_blob, d_off, d_len, d_dig)
    return d_dig


def _reduce_mod_n(x: torch.Tensor) -> torch.Tensor:
    """Values >= n (probability ~2^-32 each) are replaced by value - n, on the host."""
    nb = torch.tensor(list(N_BYTES), dtype=torch.uint8, device=x.device)
    # lexicographic compare of big-endian rows against n
    diff = x.to(torch.int16) - nb.to(torch.int16)
    first = torch.argmax((diff != 0).to(torch.int8), dim=1)
    sign = diff.gather(1, first[:, None]).squeeze(1)
    ge = sign >= 0
    if bool(ge.any()):
        for i in torch.nonzero(ge).flatten().tolist():
            v = (int.from_bytes(bytes(x[i].tolist()), "big") - int.from_bytes(N_BYTES, "big"))
            x[i] = torch.tensor(list(v.to_bytes(32, "big")), dtype=torch.uint8, device=x.device)
    return x


class Workload:
    """Device-resident SoA tuples + the expected verdicts implied by construction."""

    def __init__(self, digest, r, s, qx, qy, corrupted: torch.Tensor, start: int):
        self.digest, self.r, self.s, self.qx, self.qy = digest, r, s, qx, qy
        self.corrupted = corrupted
        self.start = start

    @property
    def n(self) -> int:
        return self.digest.shape[0]

    def host_fields(self, lo: int = 0, hi: int | None = None):
        sl = slice(lo, hi)
        return [t[sl].cpu().numpy() for t in (self.digest, self.r, self.s, self.qx, self.qy)]


def make_workload(gv, n: int, start: int = 0, device: int = 0, corrupt: bool = True) -> Workload:
    dev = torch.device(f"cuda:{device}")
    d = _reduce_mod_n(_gpu_sha(gv, *_tag_messages(b"key", start, n), dev))
    k = _reduce_mod_n(_gpu_sha(gv, *_tag_messages(b"k", start, n), dev))
    m1 = _gpu_sha(gv, *_tag_messages(b"msg", start, n), dev)
    m2 = _gpu_sha(gv, *_tag_messages(b"ms2", start, n), dev)
    msg = torch.cat([m1, m2], dim=1).contiguous()  # 64-byte messages
    blob = msg.reshape(-1).cpu().numpy()
    e = _gpu_sha(gv, blob, np.arange(n, dtype=np.uint64) * 64, np.full(n, 64, dtype=np.uint32), dev)
    qx = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    qy, r, s = torch.empty_like(qx), torch.empty_like(qx), torch.empty_like(qx)
    st = torch.empty(n, dtype=torch.uint8, device=dev)
    gv.sign_dev(d, k, e, qx, qy, r, s, st)
    torch.cuda.synchronize(dev)
    if not bool((st == 1).all()):
        raise RuntimeError(f"signer rejected {int((st != 1).sum())} synthetic keys/nonces")
    c = _gpu_sha(gv, *_tag_messages(b"c", start, n), dev)
    corrupted = c[:, 0] < 26 if corrupt else torch.zeros(n, dtype=torch.bool, device=dev)
    if corrupt:
        idx = torch.nonzero(corrupted).flatten()
        kind = (idx + start) % 7
        byte = (c[idx, 1] % 32).long()
        bit = (1 << (c[idx, 2] % 8).to(torch.int32)).to(torch.uint8)
        for kk, t in ((0, r), (1, s), (2, e)):
            sel = idx[kind == kk]
            if sel.numel():
                b = byte[kind == kk]
                t[sel, b] ^= bit[kind == kk]
        sel = idx[kind == 3]
        r[sel] = 0
        sel = idx[kind == 4]
        s[sel] = torch.tensor(list(N_BYTES), dtype=torch.uint8, device=dev)
        sel = idx[kind == 5]
        qy[sel, 31] ^= 1
        sel = idx[kind == 6]
        nb = (sel + 1) % n
        qx_nb, qy_nb = qx[nb].clone(), qy[nb].clone()
        qx[sel] = qx_nb
        qy[sel] = qy_nb
        # a neighbour that is itself replaced keeps its own original key: equal keys would
        # make the swap a no-op only if two tuples shared d, which distinct hashes exclude.
    torch.cuda.synchronize(dev)
    return Workload(e, r, s, qx, qy, corrupted, start)


def make_signed_requests(gv, n: int, start: int = 0, device: int = 0) -> list[bytes]:
    """BASELINE config 3 requests in the engine's signed-request format (include/sbft_verifier.h):
    distinct client key per request, seeded 64-256 B payloads, signed on the GPU. Request i:
    client_id "client<i>", req_id "tx<i>", payload = SHA-256 stream of seed|"pl"|le64(i)."""
    import hashlib
    dev = torch.device(f"cuda:{device}")
    d = _reduce_mod_n(_gpu_sha(gv, *_tag_messages(b"rkey", start, n), dev))
    k = _reduce_mod_n(_gpu_sha(gv, *_tag_messages(b"rk", start, n), dev))
    zero = torch.zeros((n, 32), dtype=torch.uint8, device=dev)
    one = zero.clone()
    one[:, 31] = 1
    qx, qy, r, s = (torch.empty_like(zero) for _ in range(4))
    st = torch.empty(n, dtype=torch.uint8, device=dev)
    gv.sign_dev(d, one, zero, qx, qy, r, s, st)  # pass 1: public keys
    torch.cuda.synchronize(dev)
    qxh, qyh = qx.cpu().numpy(), qy.cpu().numpy()
    rng = np.random.default_rng(start + 12345)
    lens = rng.integers(64, 257, size=n)
    bodies = []
    for i in range(n):
        cid, rid = f"client{start + i}".encode(), f"tx{start + i}".encode()
        pl = (hashlib.sha256(SEED + b"pl" + int(start + i).to_bytes(8, "little")).digest() * 9)[:lens[i]]
        bodies.append(b"SBR1" + len(cid).to_bytes(2, "little") + cid + len(rid).to_bytes(2, "little") + rid +
                      len(pl).to_bytes(4, "little") + pl + b"\x04" + qxh[i].tobytes() + qyh[i].tobytes())
    ln = np.array([len(b) for b in bodies], dtype=np.uint32)
    off = np.concatenate([[0], np.cumsum(ln)[:-1]]).astype(np.uint64)
    e = torch.from_numpy(gv.sha256(np.frombuffer(b"".join(bodies), dtype=np.uint8), off, ln)).to(dev)
    gv.sign_dev(d, k, e, qx, qy, r, s, st)  # pass 2: signatures over SHA-256(body)
    torch.cuda.synchronize(dev)
    if not bool((st == 1).all()):
        raise RuntimeError("signer rejected a synthetic request key")
    rh, sh = r.cpu().numpy(), s.cpu().numpy()
    return [bodies[i] + rh[i].tobytes() + sh[i].tobytes() for i in range(n)]


class Config5:
    """BASELINE config 5 on one device: n requests with payload lengths uniform in
    [1 KiB, 64 KiB] (seeded), resident in HBM, each signed over SHA-256 of its payload under a
    key of its own; ~10% corrupted after signing (by kind = i mod 3: an r bit, an s bit, one
    payload byte)."""

    def __init__(self, blob, off, ln, d_off, d_len, r, s, qx, qy, corrupted, total):
        self.blob, self.off, self.ln, self.d_off, self.d_len = blob, off, ln, d_off, d_len
        self.r, self.s, self.qx, self.qy, self.corrupted, self.total = r, s, qx, qy, corrupted, total

    @property
    def n(self) -> int:
        return len(self.off)


def make_config5(gv, n: int, device: int = 0, seed: int = 5) -> Config5:
    dev = torch.device(f"cuda:{device}")
    rng = np.random.default_rng(seed)
    ln = rng.integers(1024, 65537, size=n).astype(np.uint32)
    off = np.concatenate([[0], np.cumsum(ln.astype(np.uint64))[:-1]]).astype(np.uint64)
    total = int(ln.astype(np.uint64).sum())
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    blob = torch.randint(0, 256, (total + 256,), dtype=torch.uint8, device=dev, generator=g)
    d_off = torch.from_numpy(off.astype(np.int64)).to(dev)
    d_len = torch.from_numpy(ln.astype(np.int32)).to(dev)
    dig = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    gv.sha256_dev(blob, d_off, d_len, dig)
    d = _reduce_mod_n(_gpu_sha(gv, *_tag_messages(b"c5key", 0, n), dev))
    k = _reduce_mod_n(_gpu_sha(gv, *_tag_messages(b"c5k", 0, n), dev))
    qx, qy, r, s = (torch.empty((n, 32), dtype=torch.uint8, device=dev) for _ in range(4))
    st = torch.empty(n, dtype=torch.uint8, device=dev)
    gv.sign_dev(d, k, dig, qx, qy, r, s, st)
    torch.cuda.synchronize(dev)
    if not bool((st == 1).all()):
        raise RuntimeError("signer rejected a synthetic config-5 key")
    del d, k, dig
    c = _gpu_sha(gv, *_tag_messages(b"c5c", 0, n), dev)
    corrupted = c[:, 0] < 26
    idx = torch.nonzero(corrupted).flatten()
    kind = idx % 3
    byte = (c[idx, 1] % 32).long()
    bit = (1 << (c[idx, 2] % 8).to(torch.int32)).to(torch.uint8)
    for kk, t in ((0, r), (1, s)):
        sel = idx[kind == kk]
        t[sel, byte[kind == kk]] ^= bit[kind == kk]
    sel = idx[kind == 2]
    pos = d_off[sel] + (c[sel, 3].long() * 256 + c[sel, 4].long()) % d_len[sel].long()
    blob[pos] ^= bit[kind == 2]
    torch.cuda.synchronize(dev)
    return Config5(blob, off, ln, d_off, d_len, r, s, qx, qy, corrupted, total)
