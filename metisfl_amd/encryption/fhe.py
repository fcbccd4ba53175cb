"""Homomorphic encryption API (reference: metisfl/encryption/pybind/
ckks_pybind.cc:15-100, the ``fhe.CKKS`` module; demos ckks_demo.py:57-122).

``CKKS`` is the native RNS-CKKS scheme (csrc/he/ckks.cc) with the reference's
Python method names: ``gen_crypto_context_and_keys``,
``get_crypto_params_files``, ``load_crypto_context_from_file``,
``load_public_key_from_file``, ``load_private_key_from_file``, ``encrypt``,
``compute_weighted_average``, ``decrypt``.

``pwa_device`` runs the private weighted average on the GPU:
the ciphertext limbs of all learners are uploaded once and one HIP kernel does
the per-limb Shoup modular multiply-accumulate; the result is byte-identical
to the host ``compute_weighted_average``.  Ciphertext byte format (own;
Palisade's is not reproducible):
    "MCK1" | u32 N | u32 nlimbs | u32 nct | f64 log2(scale) | u64 q[nlimbs]
    | nct x {c0[nlimbs][N], c1[nlimbs][N]}
"""
from __future__ import annotations

import struct

import numpy as np

from metisfl_amd._engine import CKKS  # noqa: F401  (re-export: the reference's fhe.CKKS)

WEIGHT_BITS = 30  # weights are round(w * 2^30) per limb (ckks.h)


def _header(ct: bytes):
    if ct[:4] != b"MCK1":
        raise ValueError("not an MCK1 ciphertext")
    n, nl, nct = struct.unpack_from("<III", ct, 4)
    (logscale,) = struct.unpack_from("<d", ct, 16)
    q = np.frombuffer(ct, dtype="<u8", count=nl, offset=24)
    return n, nl, nct, logscale, q, 24 + 8 * nl


def pwa_device(ciphertexts: list[bytes], weights: list[float], device="cuda") -> bytes:
    """sum_i round(w_i * 2^30) * ct_i (mod q_j), on the GPU."""
    import torch

    from metisfl_amd.ops._native import ops
    if not ciphertexts or len(ciphertexts) != len(weights):
        raise ValueError("bad PWA inputs")
    heads = [_header(c) for c in ciphertexts]
    n, nl, nct, logscale, q, hdr = heads[0]
    for h in heads[1:]:
        if h[:4] != (n, nl, nct, logscale) or not np.array_equal(h[4], q):
            raise ValueError("ciphertexts have different parameters")
    total = nct * 2 * nl * n
    bodies = [torch.from_numpy(np.frombuffer(c, dtype="<i8", count=total, offset=hdr).copy()).to(device)
              for c in ciphertexts]
    wq = np.zeros((len(weights), nl, 2), dtype=np.uint64)
    for i, w in enumerate(weights):
        wi = int(round(float(w) * (1 << WEIGHT_BITS)))
        for j, qj in enumerate(q.tolist()):
            r = wi % qj
            wq[i, j, 0] = r
            wq[i, j, 1] = (r << 64) // qj  # Shoup precomputation
    ptrs = torch.tensor([b.data_ptr() for b in bodies], dtype=torch.int64, device=device)
    out = torch.empty(total, dtype=torch.int64, device=device)
    ops().ckks_pwa(ptrs, torch.from_numpy(wq.view(np.int64).reshape(-1)).to(device), out,
                   torch.from_numpy(q.astype(np.uint64).view(np.int64)).to(device), nl, n, nct)
    head = b"MCK1" + struct.pack("<IIId", n, nl, nct, logscale + WEIGHT_BITS) + q.astype("<u8").tobytes()
    return head + out.cpu().numpy().astype("<i8").tobytes()
