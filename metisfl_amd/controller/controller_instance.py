"""Controller process wrapper (reference:
metisfl/controller/controller_instance.py:9-51 and the pybind
ControllerWrapper, controller_pybind.cc:16-68).

Starts the gRPC servicer around the native engine, then ``shutdown()``
blocks polling (10 ms) for SIGINT/SIGTERM or a ShutDown RPC."""
from __future__ import annotations

import signal
import threading
import time

from metisfl_amd.controller.servicer import ControllerServicer
from metisfl_amd.proto import metis_pb2


class ControllerInstance:
    def __init__(self):
        self.servicer: ControllerServicer | None = None
        self._signal = False

    def start(self, controller_params_pb, checkpoint_dir: str | None = None) -> int:
        """``checkpoint_dir``: snapshot the engine there after every round /
        membership change and resume from it when it already holds one."""
        assert isinstance(controller_params_pb, metis_pb2.ControllerParams)
        self.servicer = ControllerServicer(controller_params_pb, checkpoint_dir=checkpoint_dir)
        return self.servicer.start()

    def shutdown(self, instantly: bool = False) -> None:
        def handler(signum, frame):
            self._signal = True

        if threading.current_thread() is threading.main_thread():
            signal.signal(signal.SIGTERM, handler)
            signal.signal(signal.SIGINT, handler)
        while True:
            if instantly or self._signal:
                self.servicer.stop()
                break
            if self.servicer.shutdown_request_received():
                self.servicer.wait()
                break
            time.sleep(0.01)
