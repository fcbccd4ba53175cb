"""In-process fake Redis (RESP2 over TCP) for the RedisModelStore tests.

The reference's Redis tests need a live server at 127.0.0.1:6379
(model_store_test.cc:364-380); none exists here, so this implements the
handful of commands the store uses: PING, RPUSH, LRANGE, DEL, FLUSHALL.
"""
from __future__ import annotations

import socket
import socketserver
import threading


def _bulk(b: bytes) -> bytes:
    return b"$" + str(len(b)).encode() + b"\r\n" + b + b"\r\n"


class _Handler(socketserver.BaseRequestHandler):
    def _read_line(self, buf):
        while b"\r\n" not in buf[0]:
            chunk = self.request.recv(65536)
            if not chunk:
                raise ConnectionError
            buf[0] += chunk
        line, rest = buf[0].split(b"\r\n", 1)
        buf[0] = rest
        return line

    def _read_n(self, buf, n):
        while len(buf[0]) < n + 2:
            chunk = self.request.recv(65536)
            if not chunk:
                raise ConnectionError
            buf[0] += chunk
        data = buf[0][:n]
        buf[0] = buf[0][n + 2:]
        return data

    def handle(self):
        store = self.server.store
        buf = [b""]
        try:
            while True:
                line = self._read_line(buf)
                assert line.startswith(b"*"), line
                args = []
                for _ in range(int(line[1:])):
                    ln = self._read_line(buf)
                    args.append(self._read_n(buf, int(ln[1:])))
                cmd = args[0].upper()
                with self.server.lock:
                    self.server.commands.append(cmd.decode())
                    if cmd == b"PING":
                        out = b"+PONG\r\n"
                    elif cmd == b"RPUSH":
                        lst = store.setdefault(args[1], [])
                        lst.extend(args[2:])
                        out = b":" + str(len(lst)).encode() + b"\r\n"
                    elif cmd == b"LRANGE":
                        lst = store.get(args[1], [])
                        a, b = int(args[2]), int(args[3])
                        sel = lst[a:] if b == -1 else lst[a:b + 1]
                        out = b"*" + str(len(sel)).encode() + b"\r\n" + b"".join(_bulk(x) for x in sel)
                    elif cmd == b"DEL":
                        n = sum(1 for k in args[1:] if store.pop(k, None) is not None)
                        out = b":" + str(n).encode() + b"\r\n"
                    elif cmd == b"FLUSHALL":
                        store.clear()
                        out = b"+OK\r\n"
                    else:
                        out = b"-ERR unknown command\r\n"
                self.request.sendall(out)
        except (ConnectionError, OSError):
            return


class FakeRedis(socketserver.ThreadingTCPServer):
    allow_reuse_address = True
    daemon_threads = True

    def __init__(self):
        super().__init__(("127.0.0.1", 0), _Handler)
        self.store: dict[bytes, list[bytes]] = {}
        self.commands: list[str] = []
        self.lock = threading.Lock()
        self.thread = threading.Thread(target=self.serve_forever, daemon=True)
        self.thread.start()

    @property
    def port(self) -> int:
        return self.server_address[1]

    def close(self):
        self.shutdown()
        self.server_close()
