"""``examples/fashionmnist.py --env`` on the CPU (gloo): the reference's
asynchronous + CKKS + PWA FashionMNIST configuration file runs as written
(host CKKS; tests/test_examples_gpu.py runs it on the device)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_fashionmnist_async_ckks_config_on_cpu(tmp_path):
    cfg = os.path.join(ROOT, "examples", "config", "fashionmnist",
                       "test_localhost_asynchronous_vanillasgd_with_fhe.yaml")
    wd = str(tmp_path / "fm")
    p = subprocess.run([sys.executable, "examples/fashionmnist.py", "--env", cfg, "--rounds", "3", "--device", "cpu",
                        "--train-size", "2000", "--workdir", wd], cwd=ROOT, capture_output=True, text=True,
                       timeout=600, env=dict(os.environ, PYTHONPATH=ROOT))
    assert p.returncode == 0, (p.stdout[-3000:], p.stderr[-3000:])
    md = json.load(open(os.path.join(wd, "experiment.json")))["federation_runtime_metadata"]["metadata"]
    assert max(int(m["global_iteration"]) for m in md) >= 3
    log = open(os.path.join(wd, "learner_localhost-1.log")).read()
    line = [l for l in log.splitlines() if l.startswith("[collective-async]")][-1]
    assert "over 10 learners on 1 ranks" in line and "secure PWA over ciphertexts" in line, line


import pytest  # noqa: E402


@pytest.mark.parametrize("cfg", ["brainage/brainage_test_localhost_synchronous.yaml",
                                 "brainage/brainage_test_localhost_centralized.yaml",
                                 "alzheimers_disease/alzheimers_disease_test_localhost_synchronous.yaml"])
def test_neuroimaging_configs_on_cpu(tmp_path, cfg):
    """The neuroimaging federation environment files (the reference's
    examples/config/brainage, alzheimers_disease) through
    examples/neuroimaging.py --env: every learner the file names trains on its
    TFRecord shard (the example's 3D CNN) for 2 rounds (gRPC plane)."""
    import yaml
    path = os.path.join(ROOT, "examples", "config", cfg)
    n = len(yaml.safe_load(open(path))["FederationEnvironment"]["Learners"])
    wd = str(tmp_path / "ni")
    p = subprocess.run([sys.executable, "examples/neuroimaging.py", "--env", path, "--rounds", "2", "--device", "cpu",
                        "--samples", "8", "--workdir", wd], cwd=ROOT, capture_output=True, text=True, timeout=600,
                       env=dict(os.environ, PYTHONPATH=ROOT))
    assert p.returncode == 0, (p.stdout[-3000:], p.stderr[-3000:])
    md = json.load(open(os.path.join(wd, "experiment.json")))["federation_runtime_metadata"]["metadata"]
    done = [len(m.get("completed_by_learner_id", [])) for m in md]
    assert done.count(n) >= 2, done
