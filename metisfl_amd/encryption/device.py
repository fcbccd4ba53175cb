"""Device (HIP) RNS-CKKS: encrypt / decrypt / secure weighted all-reduce on MI355X.

The reference's learners encrypt their model with Palisade CKKS on the CPU
(metisfl/encryption/palisade/ckks_scheme.cc:109-162) and the controller
computes the private weighted average over the ciphertexts
(aggregation/private_weighted_average.cc:24-82, ckks_scheme.cc:164-206);
learners decrypt the community model (ckks_scheme.cc:208-251).  Here all of
that runs on the GPU (kernels/ckks.hip: K10 NTT / canonical-embedding FFT,
K11 sampling, K9 modular scaling) over the *host scheme's* keys, twiddles and
byte layout, so a device ciphertext decrypts on the host and vice versa.

``DeviceCKKS(scheme)`` wraps a loaded ``fhe.CKKS`` (context + public key, and
the private key where the learner holds it -- the reference shares one key
pair among all learners, driver_session.py:122-135).

Secure collective aggregation (``secure_weighted_allreduce``): every rank
encrypts its flat model, multiplies its ciphertext by round(w_i * 2^30) mod
q_j, and ONE int64 sum all-reduce (RCCL over xGMI) adds the ciphertexts --
residues are < 2^60, so up to 16 addends cannot wrap 2^64 -- followed by a
mod-q reduction.  Every rank then holds Enc(sum_i w_i theta_i) and decrypts
it; plaintext models never leave their GPU.
"""
from __future__ import annotations

import math
import secrets
import struct

import numpy as np
import torch

from metisfl_amd.encryption.fhe import WEIGHT_BITS

MAX_LIMBS = 4
MAX_ALLREDUCE_RANKS = 16


def _ops():
    from metisfl_amd.ops._native import ops
    return ops()


def _shoup(w: np.ndarray, q: int) -> np.ndarray:
    return np.array([(int(x) << 64) // q for x in w.tolist()], dtype=np.uint64)


def _dev_u64(a: np.ndarray, dev) -> torch.Tensor:
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint64).view(np.int64)).to(dev)


class DeviceCKKS:
    """Device tables of one CKKS key set + the encrypt / decrypt / PWA launches."""

    def __init__(self, scheme, device="cuda"):
        self.scheme = scheme
        self.device = torch.device(device)
        t = scheme.device_tables()
        q = [int(x) for x in t["moduli"].tolist()]
        self.q = q
        self.L = len(q)
        self.N = int(scheme.ring_dim)
        self.S = int(scheme.slots)
        self.bits = int(scheme.scaling_bits)
        if self.L > MAX_LIMBS:
            raise ValueError(f"at most {MAX_LIMBS} RNS limbs on the device path")
        N, L, dev = self.N, self.L, self.device

        def per_limb_shoup(a):
            a = a.reshape(L, -1)
            return np.concatenate([_shoup(a[l], q[l]) for l in range(L)])

        garner = np.zeros((MAX_LIMBS, MAX_LIMBS, 2), dtype=np.uint64)
        for i in range(L):
            for j in range(i + 1, L):
                inv = pow(q[i] % q[j], -1, q[j])
                garner[i, j] = (inv, (inv << 64) // q[j])
        empty = torch.empty(0, dtype=torch.int64, device=dev)
        has_pk, has_sk = "pk_b" in t, "sk" in t
        self.has_public_key, self.has_private_key = has_pk, has_sk
        self.tables = [
            _dev_u64(np.array(q, dtype=np.uint64), dev),
            _dev_u64(np.array([(1 << 64) // x for x in q], dtype=np.uint64), dev),
            _dev_u64(t["psi"], dev), _dev_u64(t["psi_shoup"], dev),
            _dev_u64(t["ipsi"], dev), _dev_u64(t["ipsi_shoup"], dev),
            _dev_u64(t["n_inv"], dev), _dev_u64(t["n_inv_shoup"], dev),
            _dev_u64(t["pk_b"], dev) if has_pk else empty,
            _dev_u64(per_limb_shoup(t["pk_b"]), dev) if has_pk else empty,
            _dev_u64(t["pk_a"], dev) if has_pk else empty,
            _dev_u64(per_limb_shoup(t["pk_a"]), dev) if has_pk else empty,
            _dev_u64(t["sk"], dev) if has_sk else empty,
            _dev_u64(per_limb_shoup(t["sk"]), dev) if has_sk else empty,
            _dev_u64(garner.reshape(-1), dev),
            torch.from_numpy(t["rot"].astype(np.int32)).to(dev),
            torch.from_numpy(np.ascontiguousarray(t["ksi_re"], dtype=np.float64)).to(dev),
            torch.from_numpy(np.ascontiguousarray(t["ksi_im"], dtype=np.float64)).to(dev),
        ]
        self._scratch = None

    # ------------------------------------------------------------------
    def num_ciphertexts(self, n: int) -> int:
        return max(1, math.ceil(n / self.S))

    def ct_numel(self, n: int) -> int:
        return self.num_ciphertexts(n) * 2 * self.L * self.N

    def _scratch_for(self, n: int) -> torch.Tensor:
        need = self.num_ciphertexts(n) * self.L * self.N
        if self._scratch is None or self._scratch.numel() < need:
            self._scratch = torch.empty(need, dtype=torch.int64, device=self.device)
        return self._scratch[:need]

    def encrypt(self, x: torch.Tensor, out: torch.Tensor | None = None, key: bytes | None = None) -> torch.Tensor:
        """fp32 [n] (device) -> ciphertext limbs int64 [nct*2*L*N] at scale 2^bits.
        The noise is ChaCha20 under a fresh secret 256-bit key from the OS
        CSPRNG (``key`` only for reproducibility tests)."""
        x = x.reshape(-1)
        if x.dtype != torch.float32:
            x = x.float()
        x = x.contiguous()
        n = x.numel()
        if out is None:
            out = torch.empty(self.ct_numel(n), dtype=torch.int64, device=self.device)
        k = secrets.token_bytes(32) if key is None else bytes(key)
        _ops().ckks_encrypt(self.tables, self.N, self.L, x, out, self._scratch_for(n),
                            float(2.0 ** self.bits), k)
        return out

    def decrypt(self, ct: torch.Tensor, n: int, log2_scale: float | None = None,
                out: torch.Tensor | None = None, dtype=torch.float32) -> torch.Tensor:
        """ciphertext limbs -> fp32 / fp64 [n]; ``log2_scale`` defaults to a fresh encryption's."""
        if out is None:
            out = torch.empty(n, dtype=dtype, device=self.device)
        ls = self.bits if log2_scale is None else log2_scale
        _ops().ckks_decrypt(self.tables, self.N, self.L, ct, self._scratch_for(n), out,
                            float(2.0 ** (-ls)))
        return out

    def weight_table(self, w: float) -> torch.Tensor:
        wi = int(round(float(w) * (1 << WEIGHT_BITS)))
        rows = []
        for qj in self.q:
            r = wi % qj
            rows += [r, (r << 64) // qj]
        return _dev_u64(np.array(rows, dtype=np.uint64), self.device)

    def scale_(self, ct: torch.Tensor, w: float) -> torch.Tensor:
        """ct *= round(w * 2^30) (mod q): one learner's term of the PWA."""
        _ops().ckks_scale(self.tables, self.N, self.L, ct, self.weight_table(w))
        return ct

    def reduce_(self, ct: torch.Tensor) -> torch.Tensor:
        _ops().ckks_reduce(self.tables, self.N, self.L, ct)
        return ct

    # ------------------------------------------------------------------
    def secure_weighted_allreduce(self, comm, flat: torch.Tensor, weight: float,
                                  ct: torch.Tensor | None = None) -> dict:
        """flat <- Dec(sum_r Enc(flat_r) * w_r) over all ranks of ``comm``; returns timings (ms)."""
        if comm.world > MAX_ALLREDUCE_RANKS:
            raise ValueError(f"the int64 ciphertext all-reduce is exact for <= {MAX_ALLREDUCE_RANKS} ranks")
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        ev[0].record()
        ct = self.encrypt(flat, out=ct)
        self.scale_(ct, weight)
        ev[1].record()
        if comm.world > 1:
            comm.all_reduce_(ct)
            self.reduce_(ct)
        ev[2].record()
        self.decrypt(ct, flat.numel(), self.bits + WEIGHT_BITS, out=flat.view(-1))
        ev[3].record()
        ev[3].synchronize()
        return {"encrypt_ms": ev[0].elapsed_time(ev[1]), "allreduce_ms": ev[1].elapsed_time(ev[2]),
                "decrypt_ms": ev[2].elapsed_time(ev[3]), "ciphertext_bytes": ct.numel() * 8}

    def secure_weighted_allreduce_many(self, comm, flats: list, weights: list, out: torch.Tensor,
                                       ct: torch.Tensor | None = None, tmp: torch.Tensor | None = None) -> dict:
        """out <- Dec(sum over every learner of every rank of Enc(flat) * w):
        the co-located learners of a GPU each encrypt their own model (the
        reference's learner-side encryption), their weighted ciphertexts are
        summed on the device (int64 limbs, reduced mod q before the
        cross-rank all-reduce), then one all-reduce of ciphertexts and one
        decryption.  Returns timings (ms)."""
        if comm.world > MAX_ALLREDUCE_RANKS:
            raise ValueError(f"the int64 ciphertext all-reduce is exact for <= {MAX_ALLREDUCE_RANKS} ranks")
        n = flats[0].numel()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        ev[0].record()
        ct = self.encrypt(flats[0], out=ct)
        self.scale_(ct, weights[0])
        for k, (x, w) in enumerate(zip(flats[1:], weights[1:]), start=1):
            tmp = self.encrypt(x, out=tmp)
            self.scale_(tmp, w)
            ct.add_(tmp)
            if k % (MAX_ALLREDUCE_RANKS - 1) == 0:
                self.reduce_(ct)  # keep the int64 sums from wrapping
        self.reduce_(ct)
        ev[1].record()
        if comm.world > 1:
            comm.all_reduce_(ct)
            self.reduce_(ct)
        ev[2].record()
        self.decrypt(ct, n, self.bits + WEIGHT_BITS, out=out.view(-1))
        ev[3].record()
        ev[3].synchronize()
        return {"encrypt_ms": ev[0].elapsed_time(ev[1]), "allreduce_ms": ev[1].elapsed_time(ev[2]),
                "decrypt_ms": ev[2].elapsed_time(ev[3]), "ciphertext_bytes": ct.numel() * 8,
                "ciphertexts_encrypted": len(flats) * self.num_ciphertexts(n)}

    # ------------------------------------------------------------------
    # host byte format (he/ckks.h): "MCK1" | u32 N | u32 L | u32 nct | f64 log2 scale | u64 q[L] | body
    def to_bytes(self, ct: torch.Tensor, log2_scale: float | None = None) -> bytes:
        nct = ct.numel() // (2 * self.L * self.N)
        ls = float(self.bits if log2_scale is None else log2_scale)
        head = b"MCK1" + struct.pack("<IIId", self.N, self.L, nct, ls) + np.array(self.q, dtype="<u8").tobytes()
        return head + ct.cpu().numpy().astype("<i8").tobytes()

    def from_bytes(self, blob: bytes) -> tuple[torch.Tensor, float]:
        if blob[:4] != b"MCK1":
            raise ValueError("not an MCK1 ciphertext")
        n, nl, nct = struct.unpack_from("<III", blob, 4)
        (ls,) = struct.unpack_from("<d", blob, 16)
        q = np.frombuffer(blob, dtype="<u8", count=nl, offset=24)
        if n != self.N or nl != self.L or [int(x) for x in q] != self.q:
            raise ValueError("ciphertext from another CKKS context")
        body = np.frombuffer(blob, dtype="<i8", count=nct * 2 * nl * n, offset=24 + 8 * nl)
        return torch.from_numpy(body.copy()).to(self.device), ls


class AcceleratedCKKS:
    """``fhe.CKKS`` whose ``encrypt`` / ``decrypt`` run on the GPU.

    Drop-in for the learner-side scheme of the gRPC path (learner/he.py): the
    ciphertext bytes are the host format, so the controller's PWA (host or
    ``pwa_device``) and any host-side decrypt are unaffected.  Inputs that are
    not exactly representable in fp32 (true float64 variables) take the host
    encoder, which keeps full double precision; decryption is fp64 on device.
    """

    def __init__(self, scheme, device="cuda"):
        self._scheme = scheme
        self._dev = DeviceCKKS(scheme, device)

    def __getattr__(self, name):
        return getattr(self._scheme, name)

    def encrypt(self, values) -> bytes:
        v = np.ascontiguousarray(values, dtype=np.float64).reshape(-1)
        f = v.astype(np.float32)
        if not np.array_equal(f.astype(np.float64), v):
            return self._scheme.encrypt(v)
        ct = self._dev.encrypt(torch.from_numpy(f).to(self._dev.device))
        return self._dev.to_bytes(ct)

    def decrypt(self, ct: bytes, n: int) -> np.ndarray:
        t, ls = self._dev.from_bytes(bytes(ct))
        return self._dev.decrypt(t, int(n), ls, dtype=torch.float64).cpu().numpy()
