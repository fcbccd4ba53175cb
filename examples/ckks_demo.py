#!/usr/bin/env python3
"""CKKS API demo: encryption, decryption and private weighted average with a
separate scheme object per operation, so each step loads only the crypto
parameters it needs (encrypt: context + public key, decrypt: context +
private key, PWA: context only).  Same cases as the reference's
metisfl/encryption/ckks_demo.py:57-122 (2 learners, 2*4096 ones and 2*4096+1
twos, scaling factors 0.5), on this framework's RNS-CKKS
(metisfl_amd.encryption.CKKS), plus the same round trip through the device
(HIP) encrypt / PWA / decrypt path when a GPU is present.

  python examples/ckks_demo.py [--crypto-dir DIR]
"""
from __future__ import annotations

import argparse
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from metisfl_amd.encryption import CKKS  # noqa: E402
from metisfl_amd.utils.metis_logger import MetisLogger  # noqa: E402


def encrypt(files, scheme, learners_data):
    scheme.load_crypto_context_from_file(files["crypto_context_file"])
    scheme.load_public_key_from_file(files["public_key_file"])
    return [scheme.encrypt(np.asarray(x, dtype=np.float64)) for x in learners_data]


def decrypt(files, scheme, cts, n):
    scheme.load_crypto_context_from_file(files["crypto_context_file"])
    scheme.load_private_key_from_file(files["private_key_file"])
    return [scheme.decrypt(ct, n) for ct in cts]


def pwa(files, scheme, cts, weights):
    scheme.load_crypto_context_from_file(files["crypto_context_file"])
    return scheme.compute_weighted_average(cts, weights)


def run_case(batch_size, bits, learners_data, weights, n, crypto_dir) -> float:
    scheme = CKKS(batch_size, bits)
    scheme.gen_crypto_context_and_keys(crypto_dir)
    files = scheme.get_crypto_params_files()
    MetisLogger.info("Crypto parameters files:")
    for k, v in files.items():
        MetisLogger.info(f"\t {k}: {v}")
    enc = encrypt(files, CKKS(batch_size, bits), learners_data)
    dec = decrypt(files, CKKS(batch_size, bits), enc, n)
    MetisLogger.info(f"Learners data decrypted (first 8): {[d[:8].round(6).tolist() for d in dec]}")
    agg = pwa(files, CKKS(batch_size, bits), enc, weights)
    out = decrypt(files, CKKS(batch_size, bits), [agg], n)[0]
    MetisLogger.info(f"Aggregated (decrypted) result (first 8): {out[:8].round(6).tolist()}")
    ref = sum(w * np.asarray(x, dtype=np.float64) for w, x in zip(weights, learners_data))
    err = float(np.abs(out - ref).max())
    MetisLogger.info(f"max |error| vs plaintext weighted average: {err:.3e}")
    try:
        import torch
        if torch.cuda.is_available():
            from metisfl_amd.encryption.device import DeviceCKKS
            full = CKKS(batch_size, bits)
            full.load_context_and_keys_from_files(files["crypto_context_file"], files["public_key_file"],
                                                  files["private_key_file"])
            dev = DeviceCKKS(full, "cuda")
            acc = None
            for w, x in zip(weights, learners_data):
                ct = dev.scale_(dev.encrypt(torch.tensor(x, dtype=torch.float32, device="cuda")), w)
                acc = ct if acc is None else acc + ct
            dev.reduce_(acc)
            out_dev = dev.decrypt(acc, n, dev.bits + 30).double().cpu().numpy()
            MetisLogger.info(f"device path max |error|: {np.abs(out_dev - ref).max():.3e}")
    except ImportError:
        pass
    return err


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--crypto-dir", default=None)
    args = ap.parse_args()
    crypto_dir = args.crypto_dir or tempfile.mkdtemp(prefix="metisfl_amd_cryptoparams_")
    batch_size, bits = 4096, 52
    worst = 0.0
    for n, value in ((2 * batch_size, 1.0), (2 * batch_size + 1, 2.0)):
        learners = [[value] * n for _ in range(2)]
        weights = [0.5, 0.5]
        MetisLogger.info(f"Original learners data (first 8): {[x[:8] for x in learners]}, weights {weights}")
        worst = max(worst, run_case(batch_size, bits, learners, weights, n, crypto_dir))
    return 0 if worst < 1e-6 else 1


if __name__ == "__main__":
    sys.exit(main())
