"""HTTP/2 behaviour of the reference client's transport against the native server.

The reference client is tonic 0.1 over h2 0.2.1 (``/root/reference/Cargo.lock:393-394``)
and opens two plaintext connections (``src/lib.rs:132-138``) that every clone
shares (``src/lib.rs:148-156``, ``examples/async.rs:29-46``).  No h2 client of
that vintage exists in this image, so a raw frame-level client here reproduces
what it puts on the wire (parity unpinned -- behaviour modelled on h2 0.2's
defaults, not captured from it):

* the connection preface + a SETTINGS frame that leaves every window at the
  RFC default (65,535 bytes) and disables push;
* request bytes start flowing immediately: the first 65,535 bytes of a 602 KB
  Predict body go out BEFORE the server's SETTINGS / WINDOW_UPDATEs are read
  (and before our SETTINGS is ACKed), in 16,384-byte DATA frames (the
  default max frame size until the server's SETTINGS arrive);
* ``te: trailers``, ``content-type: application/grpc``, ``grpc-timeout``,
  ``user-agent: tonic/0.1.1`` request headers;
* its own receive window stays at 65,535 and is replenished by WINDOW_UPDATE
  only as data is consumed (h2 releases capacity once half the window is
  used), so a 602 KB response must be paced by the server's flow control
  (the client fails the test on any window overrun);
* several concurrent streams per connection, two connections in parallel.

Header blocks from the server are decoded with libnghttp2's HPACK inflater
(ctypes); everything else -- framing, windows, ordering -- is this file's.
"""
import ctypes
import socket
import struct
import threading

import numpy as np
import pytest

from rust_tensorflow_serving2_amd import _C, _build, native
from rust_tensorflow_serving2_amd.schema import serving
from rust_tensorflow_serving2_amd.utils import tensors as T

PREDICT = "/tensorflow.serving.PredictionService/Predict"
ROW = 224 * 224 * 3            # the reference's image input: 602,112 bytes of f32 per row

DATA, HEADERS, RST, SETTINGS, PING, GOAWAY, WINDOW_UPDATE, CONTINUATION = 0, 1, 3, 4, 6, 7, 8, 9
END_STREAM, END_HEADERS, ACK = 0x1, 0x4, 0x1
DEFAULT_WINDOW = 65535


# ------------------------------------------------------------------ HPACK
class _NV(ctypes.Structure):
    _fields_ = [("name", ctypes.c_void_p), ("value", ctypes.c_void_p), ("namelen", ctypes.c_size_t),
                ("valuelen", ctypes.c_size_t), ("flags", ctypes.c_uint8)]


_LIB = ctypes.CDLL(_build._nghttp2_lib())
_LIB.nghttp2_hd_inflate_new.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
_LIB.nghttp2_hd_inflate_hd2.argtypes = [ctypes.c_void_p, ctypes.POINTER(_NV), ctypes.POINTER(ctypes.c_int),
                                        ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int]
_LIB.nghttp2_hd_inflate_hd2.restype = ctypes.c_ssize_t
_LIB.nghttp2_hd_inflate_end_headers.argtypes = [ctypes.c_void_p]
_LIB.nghttp2_hd_inflate_del.argtypes = [ctypes.c_void_p]


class Inflater:
    def __init__(self):
        self.h = ctypes.c_void_p()
        assert _LIB.nghttp2_hd_inflate_new(ctypes.byref(self.h)) == 0

    def decode(self, block: bytes):
        out, off = [], 0
        buf = ctypes.create_string_buffer(block, len(block))
        base = ctypes.addressof(buf)
        while True:
            nv, flags = _NV(), ctypes.c_int(0)
            rv = _LIB.nghttp2_hd_inflate_hd2(self.h, ctypes.byref(nv), ctypes.byref(flags),
                                             ctypes.c_char_p(base + off), len(block) - off, 1)
            assert rv >= 0, f"HPACK decode error {rv}"
            off += rv
            if flags.value & 0x02:
                out.append((ctypes.string_at(nv.name, nv.namelen).decode(),
                            ctypes.string_at(nv.value, nv.valuelen).decode()))
            if flags.value & 0x01:
                _LIB.nghttp2_hd_inflate_end_headers(self.h)
                return out

    def close(self):
        _LIB.nghttp2_hd_inflate_del(self.h)


def _hpack_int(v: int, prefix: int, first: int = 0) -> bytes:
    lim = (1 << prefix) - 1
    if v < lim:
        return bytes([first | v])
    out = [first | lim]
    v -= lim
    while v >= 128:
        out.append((v & 127) | 128)
        v >>= 7
    out.append(v)
    return bytes(out)


def hpack_encode(headers) -> bytes:
    """Literal header fields without indexing, no Huffman (valid HPACK for any decoder)."""
    out = b""
    for k, v in headers:
        k, v = k.encode(), v.encode()
        out += b"\x00" + _hpack_int(len(k), 7) + k + _hpack_int(len(v), 7) + v
    return out


# ------------------------------------------------------------------ client
def frame(ftype, flags, sid, payload=b""):
    return struct.pack(">I", len(payload))[1:] + bytes([ftype, flags]) + struct.pack(">I", sid) + payload


class H2Client:
    """One connection, h2-0.2-like flow control (see the module docstring)."""

    def __init__(self, port):
        self.sock = socket.create_connection(("127.0.0.1", port), timeout=30)
        self.sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        self.inf = Inflater()
        self.send_conn = DEFAULT_WINDOW          # what the server lets us send
        self.peer_initial = DEFAULT_WINDOW
        self.peer_max_frame = 16384
        self.recv_conn = DEFAULT_WINDOW          # what we let the server send
        self.unacked_conn = 0
        self.settings_acked = False
        self.got_server_settings = False
        self.early_bytes = None                  # request bytes sent before any server frame was read
        self.streams = {}
        self.next_sid = 1
        self.rbuf = b""
        self.sock.sendall(b"PRI * HTTP/2.0\r\n\r\nSM\r\n\r\n" +
                          frame(SETTINGS, 0, 0, struct.pack(">HI", 0x2, 0)))   # ENABLE_PUSH = 0

    def open(self, body: bytes, timeout: str = "5S", path: str = PREDICT):
        sid = self.next_sid
        self.next_sid += 2
        hdrs = [(":method", "POST"), (":scheme", "http"), (":path", path), (":authority", "127.0.0.1"),
                ("content-type", "application/grpc"), ("user-agent", "tonic/0.1.1"), ("te", "trailers")]
        if timeout:
            hdrs.append(("grpc-timeout", timeout))
        self.sock.sendall(frame(HEADERS, END_HEADERS, sid, hpack_encode(hdrs)))
        msg = b"\x00" + struct.pack(">I", len(body)) + body
        self.streams[sid] = dict(out=msg, off=0, send=self.peer_initial, recv=DEFAULT_WINDOW, unacked=0,
                                 headers=None, data=b"", trailers=None, done=False, rst=None, blocks=b"")
        return sid

    def _pump_send(self):
        sent = 0
        for sid, st in self.streams.items():
            while st["off"] < len(st["out"]):
                n = min(len(st["out"]) - st["off"], self.send_conn, st["send"], self.peer_max_frame)
                if n <= 0:
                    break
                last = st["off"] + n == len(st["out"])
                self.sock.sendall(frame(DATA, END_STREAM if last else 0, sid, st["out"][st["off"]:st["off"] + n]))
                st["off"] += n
                st["send"] -= n
                self.send_conn -= n
                sent += n
        return sent

    def _read_frame(self):
        while len(self.rbuf) < 9:
            chunk = self.sock.recv(1 << 20)
            assert chunk, "server closed the connection"
            self.rbuf += chunk
        ln = int.from_bytes(self.rbuf[:3], "big")
        while len(self.rbuf) < 9 + ln:
            chunk = self.sock.recv(1 << 20)
            assert chunk, "server closed the connection"
            self.rbuf += chunk
        ftype, flags = self.rbuf[3], self.rbuf[4]
        sid = struct.unpack(">I", self.rbuf[5:9])[0] & 0x7FFFFFFF
        payload = self.rbuf[9:9 + ln]
        self.rbuf = self.rbuf[9 + ln:]
        return ftype, flags, sid, payload

    def _on_data(self, sid, flags, payload):
        n = len(payload)
        assert n <= self.recv_conn, "server overran the connection window"
        self.recv_conn -= n
        st = self.streams[sid]
        assert n <= st["recv"], f"server overran stream {sid}'s window"
        st["recv"] -= n
        st["data"] += payload
        # h2 releases capacity as the application reads; WINDOW_UPDATE once half the window is used
        self.unacked_conn += n
        st["unacked"] += n
        out = b""
        if self.unacked_conn >= DEFAULT_WINDOW // 2:
            out += frame(WINDOW_UPDATE, 0, 0, struct.pack(">I", self.unacked_conn))
            self.recv_conn += self.unacked_conn
            self.unacked_conn = 0
        if st["unacked"] >= DEFAULT_WINDOW // 2 and not flags & END_STREAM:
            out += frame(WINDOW_UPDATE, 0, sid, struct.pack(">I", st["unacked"]))
            st["recv"] += st["unacked"]
            st["unacked"] = 0
        if out:
            self.sock.sendall(out)
        if flags & END_STREAM:
            st["done"] = True

    def run(self):
        """Drive every open stream to completion; returns {sid: stream state}."""
        self.early_bytes = self._pump_send()        # before reading a single server frame
        while not all(st["done"] for st in self.streams.values()):
            ftype, flags, sid, payload = self._read_frame()
            if ftype == SETTINGS:
                if flags & ACK:
                    self.settings_acked = True
                else:
                    self.got_server_settings = True
                    for i in range(0, len(payload), 6):
                        k, v = struct.unpack(">HI", payload[i:i + 6])
                        if k == 0x4:                  # INITIAL_WINDOW_SIZE: applies to open streams too
                            for st in self.streams.values():
                                st["send"] += v - self.peer_initial
                            self.peer_initial = v
                        elif k == 0x5:
                            self.peer_max_frame = v
                    self.sock.sendall(frame(SETTINGS, ACK, 0))
            elif ftype == WINDOW_UPDATE:
                inc = struct.unpack(">I", payload)[0] & 0x7FFFFFFF
                if sid == 0:
                    self.send_conn += inc
                elif sid in self.streams:
                    self.streams[sid]["send"] += inc
            elif ftype == PING:
                if not flags & ACK:
                    self.sock.sendall(frame(PING, ACK, 0, payload))
            elif ftype == GOAWAY:
                raise AssertionError(f"GOAWAY {payload!r}")
            elif ftype in (HEADERS, CONTINUATION):
                st = self.streams[sid]
                if ftype == HEADERS and flags & 0x20:     # PRIORITY
                    payload = payload[5:]
                st["blocks"] += payload
                if ftype == HEADERS:
                    st["hflags"] = flags
                if flags & END_HEADERS:
                    hs = dict(self.inf.decode(st["blocks"]))
                    st["blocks"] = b""
                    if st["headers"] is None:
                        st["headers"] = hs
                    else:
                        st["trailers"] = hs
                    if st["hflags"] & END_STREAM:
                        st["done"] = True
            elif ftype == DATA:
                self._on_data(sid, flags, payload)
            elif ftype == RST:
                st = self.streams[sid]
                st["rst"] = struct.unpack(">I", payload)[0]
                st["done"] = True
            self._pump_send()
        return self.streams

    def close(self):
        self.inf.close()
        self.sock.close()


def grpc_status(st):
    """(status, message) from the trailers, or from a trailers-only response."""
    tr = st["trailers"] if st["trailers"] is not None else st["headers"]
    return int(tr["grpc-status"]), tr.get("grpc-message", "")


def grpc_message(st) -> bytes:
    d = st["data"]
    assert d[0] == 0
    n = struct.unpack(">I", d[1:5])[0]
    assert len(d) == 5 + n
    return d[5:]


# ------------------------------------------------------------------ server
@pytest.fixture()
def server():
    """Fast-path endpoint for [n, 224, 224, 3] f32 'images' (y = 2x + 1) served by
    a Python lane, and the Python slow path for everything else."""
    srv = _C.Http2Server("127.0.0.1", 0, 2)
    ep = srv.add_endpoint("resnet", 1, "serving_default", [("input", T.DT_FLOAT, [224, 224, 3])],
                          [("y", T.DT_FLOAT, [224, 224, 3])], 4, 1000)
    bufs = []
    for k in range(2):
        xin, yout = np.zeros((4, ROW), np.float32), np.zeros((4, ROW), np.float32)
        srv.set_slot_buffers(ep, k, [xin.ctypes.data], [yout.ctypes.data])
        bufs.append((xin, yout))
    srv.set_route("resnet", "serving_default", -1, ep)
    srv.set_route("resnet", "serving_default", 1, ep)
    stop = threading.Event()

    def lane(k):
        xin, yout = bufs[k]
        while not stop.is_set():
            n = srv.acquire(ep, k, 50)
            if n < 0:
                return
            if n:
                yout[:n] = xin[:n] * 2 + 1
                srv.complete(ep, k)

    def slow():
        while not stop.is_set():
            c = srv.next_call(50)
            if c is not None:
                srv.respond(c, 5, "Servable not found for request: Latest(nope)", b"")

    ts = [threading.Thread(target=lane, args=(k,), daemon=True) for k in range(2)] + \
        [threading.Thread(target=slow, daemon=True)]
    srv.start()
    for t in ts:
        t.start()
    yield srv
    stop.set()
    srv.remove_endpoint(ep)
    for t in ts:
        t.join(timeout=5)
    srv.stop()


def _image_request(seed, version=None):
    x = np.random.default_rng(seed).random((1, 224, 224, 3), dtype=np.float32)
    # the reference's encoding: packed float_val under "input" (src/lib.rs:237-263)
    return x, native.encode_predict_request(native.spec_tuple("resnet", version, None, "serving_default"),
                                            {"input": x}, use_tensor_content=False)


def test_602kb_predict_with_default_windows(server):
    x, body = _image_request(0)
    assert len(body) > 602112
    c = H2Client(server.port)
    try:
        sid = c.open(body)
        st = c.run()[sid]
        # the first window's worth went out before any server frame was read
        assert c.early_bytes == DEFAULT_WINDOW
        assert c.got_server_settings and c.settings_acked
        assert st["headers"][":status"] == "200" and st["headers"]["content-type"] == "application/grpc"
        assert grpc_status(st) == (0, "")
        resp = serving.PredictResponse.FromString(grpc_message(st))
        y = T.tensor_proto_to_numpy(resp.outputs["y"])
        np.testing.assert_allclose(y.reshape(1, -1), x.reshape(1, -1) * 2 + 1, rtol=1e-6)
        assert len(st["data"]) > 600000           # a 602 KB response paced by OUR 65,535-byte window
    finally:
        c.close()
    assert server.stats()["fast_path"] == 1


def test_two_connections_concurrent_streams(server):
    """The reference client's pattern: two connections shared by concurrent
    calls (examples/async.rs fan-out), several streams in flight on each."""
    results = {}

    def conn(k):
        c = H2Client(server.port)
        try:
            reqs = {}
            for i in range(4):
                x, body = _image_request(10 * k + i, version=1 if i % 2 else None)
                reqs[c.open(body)] = x
            streams = c.run()
            for sid, x in reqs.items():
                st = streams[sid]
                assert grpc_status(st) == (0, "")
                y = T.tensor_proto_to_numpy(serving.PredictResponse.FromString(grpc_message(st)).outputs["y"])
                np.testing.assert_allclose(y.reshape(-1), x.reshape(-1) * 2 + 1, rtol=1e-6)
            results[k] = len(reqs)
        finally:
            c.close()

    ts = [threading.Thread(target=conn, args=(k,)) for k in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    assert results == {0: 4, 1: 4}
    st = server.stats()
    assert st["connections"] >= 2 and st["fast_path"] == 8


def test_grpc_timeout_and_trailers_only_errors(server):
    c = H2Client(server.port)
    try:
        _x, body = _image_request(3)
        expired = c.open(body, timeout="1u")           # 1 microsecond: gone before the batch runs
        missing = c.open(native.encode_predict_request(native.spec_tuple("nope", None, None, ""),
                                                       {"x": np.zeros((1, 1), np.float32)}))
        ok = c.open(native.encode_predict_request(native.spec_tuple("resnet", None, None, ""),
                                                  {"input": np.zeros((1, 224, 224, 3), np.float32)},
                                                  use_tensor_content=True), timeout="30S")
        streams = c.run()
        assert grpc_status(streams[expired])[0] == 4                   # DEADLINE_EXCEEDED
        code, msg = grpc_status(streams[missing])
        assert code == 5 and "nope" in msg                              # NOT_FOUND, trailers-only
        assert streams[missing]["trailers"] is None and streams[missing]["data"] == b""
        assert grpc_status(streams[ok]) == (0, "")
    finally:
        c.close()
