"""Homomorphic encryption (reference: metisfl/encryption): ``fhe.CKKS`` and
the device-side private weighted average."""
from metisfl_amd.encryption.fhe import CKKS, pwa_device  # noqa: F401
