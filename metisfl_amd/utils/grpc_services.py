"""gRPC plumbing shared by every control-plane client and server
(reference: metisfl/utils/grpc_services.py:15-107).

* Unlimited message sizes both ways (models travel inside messages on the
  remote path).
* TLS when the ServerEntity's SSLConfig enables it: servers use their
  certificate + key, clients trust the peer's public certificate.
* ``request_with_timeout`` retries a call, sleeping between attempts while
  the peer is UNAVAILABLE (the reference sleeps a fixed 10 s; the back-off
  here is configurable and defaults to 10 s as well).
* Clients run requests on a small thread pool so callers can choose
  blocking or fire-and-forget (the reference uses pebble ThreadPools, which
  are not installed; concurrent.futures gives the same semantics).
"""
from __future__ import annotations

import queue
import threading
from concurrent import futures

import grpc

from metisfl_amd.utils.metis_logger import MetisLogger
from metisfl_amd.utils.ssl_configurator import SSLConfigurator

MAX_MSG_OPTIONS = [("grpc.max_send_message_length", -1),
                   ("grpc.max_receive_message_length", -1)]
# Client channels reconnect within ~2 s of a peer coming back (gRPC's default
# back-off grows to 120 s, so after a controller restart a learner's channel
# could stay in TRANSIENT_FAILURE long after the new controller listens).
CLIENT_OPTIONS = MAX_MSG_OPTIONS + [("grpc.initial_reconnect_backoff_ms", 200),
                                    ("grpc.min_reconnect_backoff_ms", 200),
                                    ("grpc.max_reconnect_backoff_ms", 2000)]


class GRPCEndpoint:
    def __init__(self, server_entity):
        self.server_entity = server_entity
        self.listening_endpoint = f"{server_entity.hostname}:{server_entity.port}"


def make_channel(server_entity) -> grpc.Channel:
    endpoint = GRPCEndpoint(server_entity).listening_endpoint
    cert, _ = SSLConfigurator.load_certificates_from_ssl_config_pb(server_entity.ssl_config, as_stream=True)
    if cert:
        return grpc.secure_channel(endpoint, grpc.ssl_channel_credentials(cert), options=CLIENT_OPTIONS)
    return grpc.insecure_channel(endpoint, options=CLIENT_OPTIONS)


class GRPCChannelMaxMsgLength:
    def __init__(self, server_entity):
        self.grpc_endpoint = GRPCEndpoint(server_entity)
        self.channel = make_channel(server_entity)


class GRPCServerClient:
    """Base of the controller / learner clients."""

    retry_sleep_s = 10.0

    def __init__(self, server_entity, max_workers: int = 1):
        self.grpc_endpoint = GRPCEndpoint(server_entity)
        self.executor = futures.ThreadPoolExecutor(max_workers=max_workers)
        self.executor_pool: "queue.Queue[futures.Future]" = queue.Queue()
        self._closing = threading.Event()
        self._channel = make_channel(server_entity)

    def get_channel(self):
        return self._channel

    # a retry cannot change these answers
    FINAL_CODES = (grpc.StatusCode.INVALID_ARGUMENT, grpc.StatusCode.NOT_FOUND, grpc.StatusCode.ALREADY_EXISTS,
                   grpc.StatusCode.PERMISSION_DENIED, grpc.StatusCode.UNAUTHENTICATED,
                   grpc.StatusCode.UNIMPLEMENTED)

    # a non-idempotent request (MarkTaskCompleted: the controller inserts the
    # model before it can fail) is retried only when it cannot have arrived,
    # or arrived and timed out (the controller drops a duplicate completion)
    TRANSIENT_CODES = (grpc.StatusCode.UNAVAILABLE, grpc.StatusCode.DEADLINE_EXCEEDED)

    def request_with_timeout(self, request_fn, request_timeout, request_retries, retry_codes=None):
        response = None
        for attempt in range(max(1, request_retries)):
            if self._closing.is_set():
                break
            try:
                return request_fn(request_timeout)
            except grpc.RpcError as err:
                MetisLogger.info("Exception raised: %s, retrying (%d/%d)...", err.code(), attempt + 1,
                                 request_retries)
                if err.code() in self.FINAL_CODES:
                    break
                if retry_codes is not None and err.code() not in retry_codes:
                    break
                if err.code() == grpc.StatusCode.UNAVAILABLE and attempt + 1 < request_retries:
                    self._closing.wait(self.retry_sleep_s)  # shutdown() cuts the back-off short
        return response

    def _schedule(self, request_fn, request_retries, request_timeout, block, retry_codes=None):
        if request_retries > 1:
            fut = self.executor.submit(self.request_with_timeout, request_fn, request_timeout, request_retries,
                                       retry_codes)
        else:
            fut = self.executor.submit(request_fn, request_timeout)
        if block:
            return fut.result()
        self.executor_pool.put(fut)
        return fut

    def cancel_retries(self):
        """Pending and future retry loops give up (no new back-off sleeps)."""
        self._closing.set()

    def shutdown(self):
        self._closing.set()
        self.executor.shutdown(wait=True)
        self._channel.close()


class GRPCServerMaxMsgLength:
    """A grpc.Server listening on the entity's endpoint (TLS if configured)."""

    def __init__(self, max_workers=None, server_entity=None):
        self.grpc_endpoint = GRPCEndpoint(server_entity)
        self.executor = futures.ThreadPoolExecutor(max_workers=max_workers)
        self.server = grpc.server(self.executor, options=MAX_MSG_OPTIONS)
        cert, key = SSLConfigurator.load_certificates_from_ssl_config_pb(server_entity.ssl_config, as_stream=True)
        if cert and key:
            creds = grpc.ssl_server_credentials(((key, cert),))
            self.port = self.server.add_secure_port(self.grpc_endpoint.listening_endpoint, creds)
        else:
            self.port = self.server.add_insecure_port(self.grpc_endpoint.listening_endpoint)
        if self.port == 0:
            raise RuntimeError(f"cannot bind {self.grpc_endpoint.listening_endpoint}")
