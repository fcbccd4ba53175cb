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


@pytest.fixture(scope="module")
def keyed(tmp_path_factory):
    from metisfl_amd.encryption import CKKS
    from metisfl_amd.encryption.device import DeviceCKKS
    from metisfl_amd.ops._native import ops
    ops()
    c = CKKS(4096, 52)
    c.gen_crypto_context_and_keys(str(tmp_path_factory.mktemp("ckks")))
    return c, DeviceCKKS(c, "cuda")


def test_device_ntt_roundtrip_and_linearity(keyed):
    """K10: forward NTT then inverse NTT is the identity on every limb."""
    import torch
    from metisfl_amd.ops._native import ops
    c, d = keyed
    rng = np.random.default_rng(1)
    rows = np.stack([rng.integers(0, q, d.N, dtype=np.uint64) for _ in range(2) for q in d.q])
    t = torch.from_numpy(rows.view(np.int64).reshape(-1).copy()).cuda()
    ops().ckks_ntt(d.tables, d.N, d.L, t, False)
    assert not torch.equal(t.cpu(), torch.from_numpy(rows.view(np.int64).reshape(-1)))
    ops().ckks_ntt(d.tables, d.N, d.L, t, True)
    assert np.array_equal(t.cpu().numpy().view(np.uint64).reshape(rows.shape), rows)


def test_device_encrypt_host_decrypt(keyed):
    """Device ciphertexts use the host byte layout, keys and twiddles."""
    import torch
    c, d = keyed
    rng = np.random.default_rng(2)
    x = rng.standard_normal(10000).astype(np.float32)
    ct = d.encrypt(torch.from_numpy(x).cuda())
    host = c.decrypt(d.to_bytes(ct), x.size)
    assert np.abs(host - x).max() < 1e-6


def test_host_encrypt_device_decrypt(keyed):
    c, d = keyed
    rng = np.random.default_rng(3)
    x = rng.standard_normal(5000)
    ct, ls = d.from_bytes(c.encrypt(x))
    out = d.decrypt(ct, x.size, ls).cpu().numpy()
    assert np.abs(out - x).max() < 1e-6


def test_device_pwa_scale_reduce_matches_weighted_mean(keyed):
    """The secure all-reduce arithmetic on one device: sum_i (w_i * ct_i mod q),
    int64 sum, mod q, decrypt == sum_i w_i x_i, and byte-identical to host PWA."""
    import torch
    c, d = keyed
    rng = np.random.default_rng(4)
    xs = [rng.standard_normal(9000).astype(np.float32) for _ in range(3)]
    w = [0.2, 0.3, 0.5]
    cts = [d.encrypt(torch.from_numpy(x).cuda()) for x in xs]
    host_pwa = c.compute_weighted_average([d.to_bytes(t) for t in cts], w)
    acc = torch.zeros_like(cts[0])
    for t, wi in zip(cts, w):
        acc += d.scale_(t.clone(), wi)
    d.reduce_(acc)
    from metisfl_amd.encryption.fhe import WEIGHT_BITS
    assert d.to_bytes(acc, d.bits + WEIGHT_BITS) == host_pwa
    out = d.decrypt(acc, 9000, d.bits + WEIGHT_BITS).cpu().numpy()
    ref = sum(wi * x.astype(np.float64) for wi, x in zip(w, xs))
    assert np.abs(out - ref).max() < 1e-5


def test_secure_allreduce_single_rank_resnet_sized(keyed):
    """Whole-model path at ResNet-18 size: Dec(Enc(theta) * 1.0) == theta."""
    import torch
    from metisfl_amd.parallel.comm import Comm
    _, d = keyed
    theta = torch.randn(11_173_962, device="cuda") * 0.05
    ref = theta.clone()
    t = d.secure_weighted_allreduce(Comm(), theta, 1.0)
    assert (theta - ref).abs().max().item() < 1e-5
    print(t)


def test_accelerated_scheme_roundtrip_through_model_codec(keyed):
    """The gRPC learner path: per-variable CiphertextTensors built by the device
    encoder decode (host PWA in between) to the weighted mean, in fp64."""
    from metisfl_amd.learner.he import accelerate
    from metisfl_amd.utils.tensor_codec import model_from_arrays, model_to_arrays
    c, _ = keyed
    acc = accelerate(c, "cuda")
    rng = np.random.default_rng(5)
    a = [rng.standard_normal((64, 33)).astype(np.float32), rng.standard_normal(10)]  # fp32 + true fp64
    b = [x * 2 for x in a]
    ma = model_from_arrays(["w", "b"], a, he_scheme=acc)
    mb = model_from_arrays(["w", "b"], b, he_scheme=acc)
    pwa = [c.compute_weighted_average([va.ciphertext_tensor.tensor_spec.value,
                                       vb.ciphertext_tensor.tensor_spec.value], [0.25, 0.75])
           for va, vb in zip(ma.variables, mb.variables)]
    for v, p in zip(ma.variables, pwa):
        v.ciphertext_tensor.tensor_spec.value = p
    _, out, _ = model_to_arrays(ma, acc)
    for o, x in zip(out, a):
        assert o.dtype == np.float64
        assert np.abs(o - 1.75 * x.astype(np.float64)).max() < 1e-6
