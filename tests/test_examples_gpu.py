"""Example federation environment files run as written on the GPU.

``examples/config/fashionmnist/test_localhost_asynchronous_vanillasgd_with_fhe.yaml``
is the reference's asynchronous + CKKS + PWA configuration
(/root/reference/examples/config/fashionmnist/, same protocol / rule /
learner count) with ``DataPlane: rccl`` and every learner on GPU 0: the
driver hosts the ten learners in one process, each encrypts on the device
after its task, rank 0 answers with the PWA over the latest ciphertexts
(parallel/async_federation.py AsyncPWA).  ``examples/fashionmnist.py --env``
runs the file; only ports, dataset paths and the round budget are set.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_fashionmnist_async_ckks_config_on_gpu(tmp_path):
    cfg = os.path.join(ROOT, "examples", "config", "fashionmnist",
                       "test_localhost_asynchronous_vanillasgd_with_fhe.yaml")
    wd = str(tmp_path / "fm")
    p = subprocess.run([sys.executable, "examples/fashionmnist.py", "--env", cfg, "--rounds", "12",
                        "--train-size", "4000", "--workdir", wd], cwd=ROOT, capture_output=True, text=True,
                       timeout=400, env=dict(os.environ, PYTHONPATH=ROOT))
    assert p.returncode == 0, (p.stdout[-3000:], p.stderr[-3000:])
    stats = json.load(open(os.path.join(wd, "experiment.json")))
    md = stats["federation_runtime_metadata"]["metadata"]
    assert max(int(m["global_iteration"]) for m in md) >= 12
    assert len({lid for m in md for lid in m.get("completed_by_learner_id", [])}) >= 2
    log = open(os.path.join(wd, "learner_localhost-1.log")).read()
    line = [l for l in log.splitlines() if l.startswith("[collective-async]")][-1]
    assert "over 10 learners on 1 ranks" in line and "secure PWA over ciphertexts" in line, line

