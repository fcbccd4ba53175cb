"""Native controller engine: aggregation numerics pinned to the reference's
gtests (federated_average_test.cc, federated_stride_test.cc,
federated_recency_test.cc, proto_tensor_serde_test.cc), scalers, CKKS."""
import numpy as np
import pytest

from metisfl_amd import _engine as E
from metisfl_amd.ops import aggregate as A
from metisfl_amd.proto import metis_pb2, model_pb2
from metisfl_amd.utils.tensor_codec import model_from_arrays, model_to_arrays, tensor_spec_to_numpy

DTYPES = [np.uint16, np.int32, np.float32, np.float64]


def _model(vals, dtype, name="var1"):
    return model_from_arrays([name], [np.asarray(vals, dtype=dtype)]).SerializeToString()


def _values(fm_bytes):
    fm = model_pb2.FederatedModel()
    fm.ParseFromString(fm_bytes)
    return model_to_arrays(fm.model)[1][0], fm


@pytest.mark.parametrize("dtype", DTYPES)
def test_fedavg_two_identical_models(dtype):
    x = np.arange(1, 11)
    m = _model(x, dtype)
    out, fm = _values(E.aggregate_models("fed_avg", [m, m], [0.5, 0.5]))
    if np.issubdtype(dtype, np.integer):
        # per-term truncation (federated_average_test.cc:106-110)
        assert out.tolist() == [0, 2, 2, 4, 4, 6, 6, 8, 8, 10]
    else:
        assert np.allclose(out, x)
    assert fm.num_contributors == 2
    assert out.dtype == np.dtype(dtype)


def test_fedavg_matches_device_kernel_semantics_host_reference():
    rng = np.random.default_rng(0)
    xs = [rng.standard_normal(1000).astype(np.float32) for _ in range(5)]
    ws = list(rng.random(5))
    out, _ = _values(E.aggregate_models("fed_avg", [_model(x, np.float32) for x in xs], ws))
    ref = A.weighted_sum_np(xs, ws)
    assert np.array_equal(out, ref)  # bit-exact: (float)((double)x*w), float adds, in order


def test_fedavg_multiple_variables_and_dtypes():
    a = model_from_arrays(["w", "b", "steps"], [np.ones((3, 4), np.float32), np.arange(4.0),
                                                np.array([4, 8], np.int64)])
    b = model_from_arrays(["w", "b", "steps"], [np.full((3, 4), 3, np.float32), np.arange(4.0) * 3,
                                                np.array([8, 16], np.int64)])
    fm = model_pb2.FederatedModel()
    fm.ParseFromString(E.aggregate_models("fed_avg", [a.SerializeToString(), b.SerializeToString()],
                                          [0.25, 0.75]))
    names, arrs, _ = model_to_arrays(fm.model)
    assert names == ["w", "b", "steps"]
    assert arrs[0].shape == (3, 4) and np.allclose(arrs[0], 2.5)
    assert np.allclose(arrs[1], np.arange(4.0) * 2.5)
    assert arrs[2].tolist() == [1 + 6, 2 + 12]


@pytest.mark.parametrize("stride", [1, 2, 3])
def test_fedstride_int32_four_learners(stride):
    x = np.arange(1, 11)
    m = _model(x, np.int32)
    out, fm = _values(E.aggregate_models("fed_stride", [m] * 4, [0.25] * 4, stride))
    if stride == 1:
        # federated_stride_test.cc:157
        assert out.tolist() == [0, 0, 0, 4, 4, 4, 4, 8, 8, 8]
    assert fm.num_contributors == 4


def test_fedstride_float_two_learners():
    a = _model(np.arange(1, 11), np.float32)
    b = _model(np.arange(1, 11) * 2, np.float32)
    out, _ = _values(E.aggregate_models("fed_stride", [a, b], [0.5, 0.5], 1))
    assert np.allclose(out, [1.5, 3.0, 4.5, 6.0, 7.5, 9.0, 10.5, 12.0, 13.5, 15.0])


def test_fedrec_rejects_longer_lineage():
    m = _model(np.arange(1, 11), np.float32)
    agg = E.FedRec()
    fm = model_pb2.FederatedModel()
    fm.ParseFromString(agg.aggregate([m, m, m], [1, 1, 1]))
    assert len(fm.model.variables) == 0


def test_fedrec_first_time_committers():
    x = np.arange(1, 11, dtype=np.float32)
    agg = E.FedRec()
    for w, vals in ((1, x), (2, x), (3, x * 0)):
        out, _ = _values(agg.aggregate([_model(vals, np.float32)], [w]))
    assert np.allclose(out, [0.5, 1, 1.5, 2, 2.5, 3, 3.5, 4, 4.5, 5])


def test_fedrec_recommit_sequence():
    # federated_recency_test.cc:238-306 -> {0.75, 1.5, ..., 7.5}
    x = np.arange(1, 11, dtype=np.float32)
    m1, m2, m3 = _model(x, np.float32), _model(x, np.float32), _model(x * 0.5, np.float32)
    agg = E.FedRec()
    seq = [([m1], [1]), ([m1], [2]), ([m1, m2], [1, 1]), ([m1, m2], [2, 2]), ([m1], [3]),
           ([m2, m3], [1, 1]), ([m2, m3], [2, 2])]
    for models, ws in seq:
        out, fm = _values(agg.aggregate(models, ws))
    assert np.allclose(out, [0.75, 1.5, 2.25, 3, 3.75, 4.5, 5.25, 6, 6.75, 7.5])
    assert fm.num_contributors == 3


@pytest.mark.parametrize("dtype", DTYPES)
def test_tensor_serde_roundtrip(dtype):
    x = (np.arange(1, 11) * 7).astype(dtype)
    m = _model(x, dtype)
    again = E.roundtrip_model(m)
    mm = model_pb2.Model()
    mm.ParseFromString(again)
    assert np.array_equal(tensor_spec_to_numpy(mm.variables[0].plaintext_tensor.tensor_spec), x)


def test_big_endian_tensor_is_normalised():
    x = np.arange(1, 6, dtype=">i4")
    m = _model(x, ">i4")
    out, _ = _values(E.aggregate_models("fed_avg", [m], [1.0]))
    assert out.tolist() == [1, 2, 3, 4, 5]


def test_quantifier_counts_zeros():
    m = _model([0, 1, 0, 2, 0], np.float32)
    assert E.quantify_model(m) == [(2, 3, 20)]


@pytest.mark.parametrize("kind,expected", [
    (3, {"a": 100 / 400, "b": 300 / 400}),   # NUM_TRAINING_EXAMPLES
    (1, {"a": 10 / 30, "b": 20 / 30}),       # NUM_COMPLETED_BATCHES
    (2, {"a": 0.5, "b": 0.5}),               # NUM_PARTICIPANTS
])
def test_scalers(kind, expected):
    got = E.scaling_factors(kind, 3, ["a", "b"], [100, 300], [10, 20])
    assert got == pytest.approx(expected)


def test_scaler_single_learner_and_single_participant_quirk():
    assert E.scaling_factors(3, 1, ["a"], [100], [10]) == {"a": 1.0}
    # one participant among many learners gets its raw value
    assert E.scaling_factors(3, 4, ["a"], [100], [10]) == {"a": 100.0}
    assert E.scaling_factors(1, 4, ["a"], [100], [10]) == {"a": 10.0}
    assert E.scaling_factors(2, 4, ["a"], [100], [10]) == {"a": 1.0}


def test_python_scaling_mirror_matches_engine():
    from metisfl_amd.parallel import scaling
    for kind, name in ((1, "NUM_COMPLETED_BATCHES"), (2, "NUM_PARTICIPANTS"), (3, "NUM_TRAINING_EXAMPLES")):
        for n_all, ids in ((1, ["a"]), (3, ["a"]), (3, ["a", "b", "c"])):
            nt = [100, 250, 650][: len(ids)]
            nb = [10, 20, 30][: len(ids)]
            e = E.scaling_factors(kind, n_all, ids, nt, nb)
            p = scaling.compute(name, nt, nb, n_all)
            assert [e[i] for i in ids] == pytest.approx(p)


# ---------------------------------------------------------------------------
def test_ckks_encrypt_pwa_decrypt(tmp_path):
    c = E.CKKS(4096, 52)
    c.gen_crypto_context_and_keys(str(tmp_path))
    files = c.get_crypto_params_files()
    for k in ("crypto_context_file", "public_key_file", "private_key_file", "eval_mult_key_file"):
        assert (tmp_path / files[k].split("/")[-1]).exists()
    a = np.array([1, 2, 2, 4, 5, 6, 7, 8, 9, 10], dtype=np.float64)
    ca, cb = c.encrypt(a), c.encrypt(a)
    # private_weighted_average_test.cc: PWA(0.5, 0.5) compared as ints
    pwa = c.compute_weighted_average([ca, cb], [0.5, 0.5])
    out = c.decrypt(pwa, len(a))
    assert np.rint(out).astype(int).tolist() == a.astype(int).tolist()
    assert np.abs(out - a).max() < 1e-6


def test_ckks_controller_side_only_needs_context(tmp_path):
    learner = E.CKKS(4096, 52)
    learner.gen_crypto_context_and_keys(str(tmp_path))
    f = learner.get_crypto_params_files()
    ctrl = E.CKKS(4096, 52)
    ctrl.load_crypto_context_from_file(f["crypto_context_file"])
    rng = np.random.default_rng(1)
    xs = [rng.standard_normal(10000) for _ in range(3)]
    cts = [learner.encrypt(x) for x in xs]
    out = learner.decrypt(ctrl.compute_weighted_average(cts, [0.2, 0.3, 0.5]), 10000)
    assert np.abs(out - (0.2 * xs[0] + 0.3 * xs[1] + 0.5 * xs[2])).max() < 1e-6
    with pytest.raises(RuntimeError):
        ctrl.decrypt(cts[0], 10)  # no private key on the controller


def test_ckks_keys_reload(tmp_path):
    a = E.CKKS(4096, 52)
    a.gen_crypto_context_and_keys(str(tmp_path))
    f = a.get_crypto_params_files()
    b = E.CKKS(4096, 52)
    b.load_context_and_keys_from_files(f["crypto_context_file"], f["public_key_file"],
                                       f["private_key_file"])
    x = np.linspace(-5, 5, 5000)
    assert np.abs(b.decrypt(a.encrypt(x), 5000) - x).max() < 1e-6
    assert np.abs(a.decrypt(b.encrypt(x), 5000) - x).max() < 1e-6


def test_encrypted_model_codec(tmp_path):
    c = E.CKKS(4096, 52)
    c.gen_crypto_context_and_keys(str(tmp_path))
    m = model_from_arrays(["w"], [np.arange(12, dtype=np.float32).reshape(3, 4)], he_scheme=c)
    assert m.variables[0].HasField("ciphertext_tensor")
    names, arrs, _ = model_to_arrays(m, he_scheme=c)
    assert arrs[0].shape == (3, 4)
    assert np.allclose(arrs[0], np.arange(12).reshape(3, 4), atol=1e-5)
