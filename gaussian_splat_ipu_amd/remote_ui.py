"""Client side of the render server's remote-UI protocol (bin/splat
--ui-port, csrc/host/remote_ui.hpp; reference: include/remote_ui/
InterfaceServer.hpp).  Packet names and their order are the reference's
(InterfaceServer.hpp:24-43); the framing is this build's own (the reference's
packetcomms library is not in the snapshot):

    packet = u32 type index | u32 payload bytes | payload   (little-endian)
"""
from __future__ import annotations

import socket
import struct
import time
import zlib

import numpy as np

PACKET_TYPES = [
    "stop", "detach", "env_rotation", "env_rotation_2", "exposure", "gamma", "X", "Y", "Z",
    "lambda1", "lambda2", "fov", "render_preview", "ready", "tile_histogram", "device",
]
_FLOAT_PACKETS = {"env_rotation", "env_rotation_2", "exposure", "gamma", "X", "Y", "Z", "lambda1", "lambda2",
                  "fov"}


class UiClient:
    def __init__(self, host: str, port: int, timeout: float = 60.0, connect_wait: float = 30.0):
        t0 = time.time()
        while True:
            try:
                self.sock = socket.create_connection((host, port), timeout=timeout)
                break
            except OSError:
                if time.time() - t0 > connect_wait:
                    raise
                time.sleep(0.05)
        self.sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        # syncWithClient(..., "ready"): both sides send it
        name, _ = self.recv()
        assert name == "ready", name
        self.send_raw("ready", b"")

    def close(self):
        self.sock.close()

    def _recv_all(self, n: int) -> bytes:
        buf = bytearray()
        while len(buf) < n:
            chunk = self.sock.recv(n - len(buf))
            if not chunk:
                raise ConnectionError("server closed the connection")
            buf += chunk
        return bytes(buf)

    def recv(self):
        """(packet name, decoded payload)."""
        t, n = struct.unpack("<II", self._recv_all(8))
        p = self._recv_all(n) if n else b""
        name = PACKET_TYPES[t] if t < len(PACKET_TYPES) else str(t)
        if name == "tile_histogram":
            (cnt,) = struct.unpack_from("<Q", p)
            return name, np.frombuffer(p, np.uint32, cnt, 8).copy()
        if name == "render_preview":
            w, h, codec = struct.unpack_from("<iiI", p)
            assert codec == 1
            return name, np.frombuffer(zlib.decompress(p[12:]), np.uint8).reshape(h, w, 3)
        if name in _FLOAT_PACKETS:
            return name, struct.unpack("<f", p)[0]
        return name, p

    def send_raw(self, name: str, payload: bytes):
        self.sock.sendall(struct.pack("<II", PACKET_TYPES.index(name), len(payload)) + payload)

    def send(self, name: str, value):
        """Client -> server state updates: floats (fov in degrees, as the
        reference UI sends it), stop/detach (bool), device (string)."""
        if name in _FLOAT_PACKETS:
            self.send_raw(name, struct.pack("<f", float(value)))
        elif name in ("stop", "detach"):
            self.send_raw(name, bytes([1 if value else 0]))
        elif name == "device":
            b = value.encode()
            self.send_raw(name, struct.pack("<Q", len(b)) + b)
        else:
            raise ValueError(name)

    def frame(self):
        """The next (histogram, preview) pair the server sends after a frame."""
        hist = img = None
        while hist is None or img is None:
            name, v = self.recv()
            if name == "tile_histogram":
                hist = v
            elif name == "render_preview":
                img = v
        return hist, img
