"""CKKS randomness: ChaCha20 (RFC 8439) on the host, known-answer vectors,
and chi-square / moment tests of the three samplers (ternary secret,
discrete Gaussian error, uniform mod q).  The device twin is
tests/test_ckks_rng_gpu.py."""
import numpy as np
from scipy import stats

RFC8439_KEY = bytes(range(32))
RFC8439_NONCE = bytes.fromhex("000000090000004a00000000")
# RFC 8439 section 2.3.2: block counter 1
RFC8439_BLOCK = bytes.fromhex(
    "10f1e7e4d13b5915500fdd1fa32071c4c7d1f4c733c068030422aa9ac3d46c4e"
    "d2826446079faa0914c2d705d98b02a2b5129cd1de164eb9cbd083e8a2503c4e")
# RFC 8439 appendix A.1 test vector #1: all-zero key / nonce, counter 0
ZERO_BLOCK = bytes.fromhex(
    "76b8e0ada0f13d90405d6ae55386bd28bdd219b8a08ded1aa836efcc8b770dc7"
    "da41597c5157488d7724e03fb8d84a376a43b8f41518a11cc387b669b2ee6586")


def _engine():
    import metisfl_amd._engine as e
    return e


def test_chacha20_known_answers_host():
    e = _engine()
    assert e.chacha20_block(RFC8439_KEY, 1, RFC8439_NONCE) == RFC8439_BLOCK
    assert e.chacha20_block(bytes(32), 0, bytes(12)) == ZERO_BLOCK


def _ckks():
    e = _engine()
    c = e.CKKS(4096, 52)
    return c


def test_ternary_sampler_uniform():
    v = np.asarray(_ckks().debug_sample(0, 300_000))
    assert set(np.unique(v)) <= {-1, 0, 1}
    counts = np.array([(v == t).sum() for t in (-1, 0, 1)])
    assert stats.chisquare(counts).pvalue > 1e-6, counts


def test_gaussian_sampler_sigma_3_2():
    v = np.asarray(_ckks().debug_sample(1, 400_000)).astype(np.float64)
    assert np.abs(v).max() <= 19
    assert abs(v.mean()) < 0.03
    assert abs(v.var() - (3.2 ** 2 + 1 / 12)) < 0.15  # rounding adds 1/12
    # chi-square against the rounded normal on |x| <= 8 (tails pooled)
    edges = np.arange(-8.5, 9.5, 1.0)
    obs, _ = np.histogram(v, bins=np.concatenate([[-np.inf], edges, [np.inf]]))
    cdf = stats.norm.cdf(np.concatenate([[-np.inf], edges, [np.inf]]), scale=3.2)
    exp = np.diff(cdf) * v.size
    assert stats.chisquare(obs, exp).pvalue > 1e-6


def test_uniform_mod_q_sampler():
    c = _ckks()
    q = c.moduli[0]
    v = np.asarray(c.debug_sample(2, 200_000), dtype=np.float64)
    assert v.min() >= 0 and v.max() < q
    obs, _ = np.histogram(v / q, bins=64, range=(0.0, 1.0))
    assert stats.chisquare(obs).pvalue > 1e-6


def test_keys_differ_between_contexts(tmp_path):
    """Two contexts draw independent keys (no shared or guessable seed)."""
    e = _engine()
    a, b = e.CKKS(4096, 52), e.CKKS(4096, 52)
    da, db = tmp_path / "a", tmp_path / "b"
    a.gen_crypto_context_and_keys(str(da))
    b.gen_crypto_context_and_keys(str(db))
    fa, fb = a.get_crypto_params_files(), b.get_crypto_params_files()
    ka = open(fa["public_key_file"], "rb").read()
    kb = open(fb["public_key_file"], "rb").read()
    assert ka != kb
    # and the same plaintext encrypts to different ciphertexts
    x = np.linspace(-1, 1, 100)
    assert a.encrypt(x) != a.encrypt(x)
