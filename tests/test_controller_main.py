"""The standalone controller executable (build/native/metisfl_controller,
reference metisfl/controller/controller_main.cc): starts with the
reference's defaults on the given port, answers the health RPC, serves a
join, and shuts down on SIGTERM."""
import os
import signal
import socket
import subprocess
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "build", "native", "metisfl_controller")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.skipif(not os.path.exists(EXE), reason="native build not present")
def test_standalone_controller_binary(tmp_path):
    from metisfl_amd.utils.grpc_controller_client import GRPCControllerClient
    from metisfl_amd.utils.proto_messages_factory import MetisProtoMessages as M
    port = _free_port()
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", METISFL_AMD_ROOT=ROOT)
    p = subprocess.Popen([EXE, "--port", str(port)], env=env, stdout=subprocess.PIPE,
                         stderr=subprocess.STDOUT, start_new_session=True)
    try:
        client = GRPCControllerClient(M.construct_server_entity_pb("127.0.0.1", port))
        deadline = time.time() + 120
        ok = False
        while time.time() < deadline and not ok:
            try:
                ok = client.check_health_status(request_timeout=2).services_status["controller"]
            except Exception:
                time.sleep(0.5)
            assert p.poll() is None, p.stdout.read().decode()
        assert ok
        assert client.shutdown_controller()
        client.shutdown()
        p.wait(timeout=60)
    finally:
        if p.poll() is None:
            os.killpg(p.pid, signal.SIGTERM)
            p.wait(timeout=30)
