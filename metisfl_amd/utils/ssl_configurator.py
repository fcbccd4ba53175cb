"""TLS material for the gRPC control plane (reference:
metisfl/utils/ssl_configurator.py:16-77, resources/ssl_config/gen_certificates.sh).

The reference ships pre-generated default certificates; here they are
generated on first use with the ``openssl`` CLI (pyOpenSSL is not
installed) into a per-user cache directory, as a self-signed server
certificate valid for localhost / 127.0.0.1 / ::1.  A learner never sends
its private key to the controller: ``gen_public_ssl_config_pb_as_stream``
strips it (reference: grpc_controller_client.py:56-70)."""
from __future__ import annotations

import os
import subprocess
import tempfile

from metisfl_amd.proto import metis_pb2
from metisfl_amd.utils.metis_logger import MetisLogger

def _default_dir() -> str:
    return os.environ.get("METISFL_AMD_SSL_DIR",
                          os.path.join(tempfile.gettempdir(), "metisfl_amd_ssl_default"))


def generate_self_signed(out_dir: str, common_name: str = "localhost", days: int = 3650):
    """Write server-cert.pem / server-key.pem (RSA-2048, SAN localhost + loopback)."""
    os.makedirs(out_dir, exist_ok=True)
    cert = os.path.join(out_dir, "server-cert.pem")
    key = os.path.join(out_dir, "server-key.pem")
    if os.path.exists(cert) and os.path.exists(key):
        return cert, key
    cfg = os.path.join(out_dir, "openssl.cnf")
    with open(cfg, "w") as f:
        f.write("[req]\ndistinguished_name=dn\nx509_extensions=ext\nprompt=no\n"
                f"[dn]\nCN={common_name}\n"
                "[ext]\nsubjectAltName=DNS:localhost,IP:127.0.0.1,IP:::1\n"
                "basicConstraints=critical,CA:TRUE\n")
    subprocess.run(["openssl", "req", "-x509", "-newkey", "rsa:2048", "-nodes", "-keyout", key,
                    "-out", cert, "-days", str(days), "-config", cfg],
                   check=True, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    os.chmod(key, 0o600)
    return cert, key


class SSLConfigurator:

    @classmethod
    def gen_default_certificates(cls, as_stream: bool = False):
        cert, key = generate_self_signed(_default_dir())
        if as_stream:
            return cls.load_file_as_stream(cert), cls.load_file_as_stream(key)
        return cert, key

    @classmethod
    def load_file_as_stream(cls, filepath):
        if filepath and os.path.exists(filepath):
            with open(filepath, "rb") as f:
                return f.read()
        return None

    @classmethod
    def load_certificates_from_ssl_config_pb(cls, ssl_config_pb, as_stream: bool = False):
        """(public_certificate, private_key) from an SSLConfig; (None, None)
        when TLS is disabled."""
        cert, key = None, None
        if ssl_config_pb is not None and ssl_config_pb.enable_ssl:
            which = ssl_config_pb.WhichOneof("config")
            if which == "ssl_config_files":
                cert = ssl_config_pb.ssl_config_files.public_certificate_file or None
                key = ssl_config_pb.ssl_config_files.private_key_file or None
                if as_stream:
                    cert, key = cls.load_file_as_stream(cert), cls.load_file_as_stream(key)
            elif which == "ssl_config_stream":
                cert = ssl_config_pb.ssl_config_stream.public_certificate_stream or None
                key = ssl_config_pb.ssl_config_stream.private_key_stream or None
            else:
                MetisLogger.warning("SSL requested but no certificate given; proceeding without SSL.")
        return cert, key

    @classmethod
    def gen_public_ssl_config_pb_as_stream(cls, ssl_config_pb):
        """Copy of ``ssl_config_pb`` holding only the public certificate bytes."""
        out = metis_pb2.SSLConfig(enable_ssl=bool(ssl_config_pb is not None and ssl_config_pb.enable_ssl))
        if out.enable_ssl:
            cert, _ = cls.load_certificates_from_ssl_config_pb(ssl_config_pb, as_stream=True)
            out.ssl_config_stream.CopyFrom(metis_pb2.SSLConfigStream(public_certificate_stream=cert or b""))
        return out

    @classmethod
    def default_ssl_config_pb(cls):
        cert, key = cls.gen_default_certificates(as_stream=False)
        return metis_pb2.SSLConfig(enable_ssl=True, ssl_config_files=metis_pb2.SSLConfigFiles(
            public_certificate_file=cert, private_key_file=key))
