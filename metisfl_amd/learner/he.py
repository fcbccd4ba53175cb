"""Homomorphic-encryption scheme factory for learners (reference:
learner.py:208-246 builds ``fhe.CKKS`` from HESchemeConfig and loads the
crypto context and keys from files).  On a GPU learner the scheme's
encrypt / decrypt run on the device (K10/K11 kernels), same bytes."""
from __future__ import annotations


def he_scheme_from_config(he_scheme_pb):
    if he_scheme_pb is None or not he_scheme_pb.enabled:
        return None
    if not he_scheme_pb.HasField("ckks_scheme_config"):
        raise ValueError("only the CKKS scheme is supported")
    from metisfl_amd import _engine
    c = he_scheme_pb.ckks_scheme_config
    scheme = _engine.CKKS(c.batch_size, c.scaling_factor_bits)
    scheme.load_crypto_context_from_file(he_scheme_pb.crypto_context_file)
    scheme.load_public_key_from_file(he_scheme_pb.public_key_file)
    if he_scheme_pb.private_key_file:
        scheme.load_private_key_from_file(he_scheme_pb.private_key_file)
    return accelerate(scheme)


def accelerate(scheme, device=None):
    """On a GPU learner, encrypt / decrypt run through the HIP CKKS kernels
    (encryption/device.py); the ciphertext bytes are unchanged."""
    import torch
    if device is None and not torch.cuda.is_available():
        return scheme
    from metisfl_amd.encryption.device import AcceleratedCKKS
    return AcceleratedCKKS(scheme, device or "cuda")
