"""The CKKS API demo (reference: metisfl/encryption/ckks_demo.py) runs end to
end on the host scheme: per-operation key loading, 2 learners, the 2*4096 and
2*4096+1 element cases, PWA within 1e-6 of the plaintext weighted mean."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_ckks_demo_runs(tmp_path):
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "examples", "ckks_demo.py"), "--crypto-dir",
                        str(tmp_path)], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    assert "Aggregated (decrypted) result" in (r.stdout + r.stderr)
    assert (tmp_path / "cryptocontext.txt").exists() and (tmp_path / "key-public.txt").exists()
