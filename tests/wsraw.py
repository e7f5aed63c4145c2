"""A raw RFC 6455 client for driving a WebSocket server byte for byte (test
helper): HTTP Upgrade handshake, then a scripted byte stream sent in chosen
chunks, and everything the server sends back collected until it closes the
connection. Server frames are parsed (unmasked, 2 / 4 / 10-byte headers).
With tls=True the same over a TLS connection (no certificate check: the
test servers use the self-signed tests/tls certificate)."""
import socket
import ssl
import struct
import time

from wsframes import frame

HANDSHAKE = (b"GET / HTTP/1.1\r\nHost: 127.0.0.1\r\nUpgrade: websocket\r\nConnection: Upgrade\r\n"
             b"Sec-WebSocket-Key: dGhlIHNhbXBsZSBub25jZQ==\r\nSec-WebSocket-Version: 13\r\n\r\n")


def connect(port, timeout=10.0, tls=False):
    s = socket.create_connection(("127.0.0.1", port), timeout=timeout)
    s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
    if tls:
        ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_CLIENT)
        ctx.check_hostname = False
        ctx.verify_mode = ssl.CERT_NONE
        s = ctx.wrap_socket(s, server_hostname="127.0.0.1")
    s.sendall(HANDSHAKE)
    reply = b""
    while b"\r\n\r\n" not in reply:
        b = s.recv(4096)
        if not b:
            raise ConnectionError("closed during handshake")
        reply += b
    head, rest = reply.split(b"\r\n\r\n", 1)
    assert head.startswith(b"HTTP/1.1 101"), head
    return s, head, rest


def run_script(port, stream, chunks, pause_s=0.0002, timeout=10.0, tls=False):
    """Send `stream` in pieces of the given sizes (over TLS: one record each),
    then read until the server closes. Returns (handshake reply head, every
    byte received after it)."""
    assert sum(chunks) == len(stream)
    s, head, got = connect(port, timeout, tls)
    pos, i = 0, 0
    try:
        while pos < len(stream):
            n = chunks[i]
            s.sendall(stream[pos:pos + n])
            pos += n
            i += 1
            if pause_s:
                time.sleep(pause_s)
    except (BrokenPipeError, ConnectionResetError, ssl.SSLError):
        pass
    s.settimeout(timeout)
    try:
        while True:
            b = s.recv(1 << 16)
            if not b:
                break
            got += b
    except (ConnectionResetError, socket.timeout, ssl.SSLError):
        pass
    s.close()
    return head, got


def parse_server_frames(data):
    """[(fin, opcode, payload)] of unmasked server frames; trailing partial bytes ignored."""
    out, p = [], 0
    while p + 2 <= len(data):
        b0, b1 = data[p], data[p + 1]
        n, h = b1 & 127, 2
        if n == 126:
            n, h = struct.unpack(">H", data[p + 2:p + 4])[0], 4
        elif n == 127:
            n, h = struct.unpack(">Q", data[p + 2:p + 10])[0], 10
        if p + h + n > len(data):
            break
        out.append((b0 >> 7, b0 & 15, data[p + h:p + h + n]))
        p += h + n
    return out


def close_frame(code, reason=b"", key=0x11223344):
    return frame(8, struct.pack(">H", code) + reason, key=key)
