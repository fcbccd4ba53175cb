"""K9: the device private weighted average (HIP kernel) is byte-identical to
the host CKKS PWA and decrypts to the weighted mean."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_pwa_device_matches_host(tmp_path):
    from metisfl_amd.encryption import CKKS, pwa_device
    from metisfl_amd.ops._native import ops
    ops()
    c = CKKS(4096, 52)
    c.gen_crypto_context_and_keys(str(tmp_path))
    rng = np.random.default_rng(0)
    xs = [rng.standard_normal(9000) for _ in range(3)]
    cts = [c.encrypt(x) for x in xs]
    w = [0.2, 0.3, 0.5]
    host = c.compute_weighted_average(cts, w)
    dev = pwa_device(cts, w)
    assert dev == host
    out = c.decrypt(dev, 9000)
    assert np.abs(out - sum(wi * x for wi, x in zip(w, xs))).max() < 1e-6
