"""ZMTP 3.x endpoints (PULL and REP, NULL mechanism) over TCP, from the published wire
protocol, so that the reference's unchanged ZeroMQ clients reach the HBM replay.

Why: a remote actor (test/apex-dqn/worker.py:21-61) builds `reth_buffer.Client(meta_addr)`,
which (reth_buffer/reth_buffer/client/client.py:9-19, utils/__init__.py:51-59) sends one REQ
to the service's meta address, reads the JSON config it returns, then PUSHes
`serialize([rows, weights])` messages to `append_addr` (client.py:21-35) -- received by the
service's PULL socket (server/main_loop.py:21-26,44-46) -- and priority updates to
`update_addr` (client.py:37-39).  pyzmq / libzmq are not in this image, so the three
sockets are written here against the protocol itself (ZMTP 3.1, rfc.zeromq.org/spec/37; ZMTP
3.0, spec/23; the NULL security mechanism), Python sockets, one thread per peer:

  greeting   64 bytes: signature FF 00*8 7F, version 3.x, mechanism "NULL" (20 bytes,
             zero-padded), as-server 0, 31 bytes of filler
  handshake  each side sends a READY command whose Socket-Type property names its socket
             type; the peer's type is checked against the valid pairs (PULL <- PUSH,
             REP <- REQ | DEALER); anything else gets an ERROR command and the connection
             is closed
  traffic    frames: a flags byte (bit 0 MORE, bit 1 LONG = 8-byte size, bit 2 COMMAND), the
             size (1 or 8 bytes, network order), the body; a message is the frames up to one
             without MORE.  PING commands are answered with PONG (their context echoed), other
             commands are ignored

A PULL endpoint hands every message (a list of frame bodies) to `on_message`, which may
block: the reader stops reading the TCP stream, so the sender's TCP window -- and then its
own send queue -- applies the back-pressure ZMQ's high-water mark does.  A REP endpoint
replies to each request with `on_request(body_frames)` under the request's envelope
(every frame up to and including the empty delimiter).

Message size: the endpoints are unauthenticated, so a frame header's 8-byte size is checked
against `max_msg_size` before any buffer is allocated (the role of ZMQ_MAXMSGSIZE; a larger
frame, or a message whose frames add up to more, closes that connection with a ZmtpError
recorded in `Endpoint.errors`).  Any other failure of one connection -- a handler raising
included -- ends that connection only; the listener and the other peers keep running."""
import fcntl
import socket
import struct
import threading

SIGNATURE = b"\xff" + b"\x00" * 8 + b"\x7f"
MORE, LONG, COMMAND = 1, 2, 4
DEFAULT_MAX_MSG_SIZE = 1 << 30  # 1 GiB: far above a worker's append message (64 Pong rows = 14.5 MB)
VALID_PEERS = {b"PULL": {b"PUSH"}, b"REP": {b"REQ", b"DEALER"}, b"PUSH": {b"PULL"}, b"REQ": {b"REP", b"ROUTER"}}


class ZmtpError(Exception):
    pass


def greeting(as_server=False, mechanism=b"NULL", minor=1):
    """the 64-byte ZMTP 3.x greeting"""
    return SIGNATURE + bytes([3, minor]) + mechanism.ljust(20, b"\x00") + bytes([1 if as_server else 0]) + b"\x00" * 31


def encode_frame(body, more=False, command=False):
    body = bytes(body)
    flags = (MORE if more else 0) | (COMMAND if command else 0)
    if len(body) > 255:
        return bytes([flags | LONG]) + struct.pack(">Q", len(body)) + body
    return bytes([flags, len(body)]) + body


def encode_message(frames):
    frames = list(frames)
    return b"".join(encode_frame(f, more=i < len(frames) - 1) for i, f in enumerate(frames))


def encode_command(name, body=b""):
    return encode_frame(bytes([len(name)]) + name + body, command=True)


def encode_properties(props):
    return b"".join(bytes([len(k)]) + k + struct.pack(">I", len(v)) + v for k, v in props)


def ready_command(socket_type, identity=None):
    props = [(b"Socket-Type", socket_type)]
    if identity is not None:
        props.append((b"Identity", identity))
    return encode_command(b"READY", encode_properties(props))


def parse_command(body):
    """(name, data) of a command frame's body"""
    if not body:
        raise ZmtpError("empty command")
    n = body[0]
    return bytes(body[1:1 + n]), bytes(body[1 + n:])


def parse_properties(data):
    props, i = {}, 0
    while i < len(data):
        n = data[i]
        name = bytes(data[i + 1:i + 1 + n])
        i += 1 + n
        if i + 4 > len(data):
            raise ZmtpError("truncated property")
        (vlen,) = struct.unpack(">I", data[i:i + 4])
        props[name.lower()] = bytes(data[i + 4:i + 4 + vlen])
        i += 4 + vlen
    return props


class Connection:
    """one accepted TCP peer: greeting + NULL handshake, then frame I/O"""

    def __init__(self, sock, socket_type, max_msg_size=None):
        self.sock = sock
        self.socket_type = socket_type
        self.peer_type = None
        self.max_msg_size = DEFAULT_MAX_MSG_SIZE if max_msg_size is None else int(max_msg_size)
        self._wlock = threading.Lock()

    def recv_exact(self, n):
        buf = bytearray(n)
        view, got = memoryview(buf), 0
        while got < n:
            k = self.sock.recv_into(view[got:], n - got)
            if k == 0:
                raise ConnectionError("peer closed the connection")
            got += k
        return buf

    def send(self, data):
        with self._wlock:
            self.sock.sendall(data)

    def handshake(self):
        self.send(greeting())
        sig = self.recv_exact(10)
        if sig[0] != 0xFF or not (sig[9] & 1):
            raise ZmtpError("not a ZMTP 3 peer (signature)")
        ver = self.recv_exact(2)
        if ver[0] < 3:
            raise ZmtpError(f"ZMTP {ver[0]}.{ver[1]} peer (3.x required)")
        rest = self.recv_exact(52)
        mech = rest[:20].rstrip(b"\x00")
        if mech != b"NULL":
            raise ZmtpError(f"security mechanism {mech!r} (only NULL)")
        self.send(ready_command(self.socket_type))
        flags, body = self.read_frame()
        if not flags & COMMAND:
            raise ZmtpError("expected READY")
        name, data = parse_command(body)
        if name == b"ERROR":
            raise ZmtpError(f"peer error: {data[1:1 + data[0]] if data else b''!r}")
        if name != b"READY":
            raise ZmtpError(f"expected READY, got {name!r}")
        self.peer_type = parse_properties(data).get(b"socket-type", b"")
        if self.peer_type not in VALID_PEERS.get(self.socket_type, ()):
            reason = b"invalid socket type " + self.peer_type
            self.send(encode_command(b"ERROR", bytes([len(reason)]) + reason))
            raise ZmtpError(f"{self.socket_type.decode()} endpoint refuses a {self.peer_type.decode()} peer")

    def read_frame(self, budget=None):
        """(flags, body); the size is checked against `budget` (default max_msg_size) before
        the body's buffer is allocated"""
        flags = self.recv_exact(1)[0]
        if flags & LONG:
            (size,) = struct.unpack(">Q", self.recv_exact(8))
        else:
            size = self.recv_exact(1)[0]
        limit = self.max_msg_size if budget is None else budget
        if size > limit:
            raise ZmtpError(f"frame of {size} bytes exceeds the message size limit ({self.max_msg_size} bytes)")
        return flags, self.recv_exact(size)

    def read_message(self):
        """the next message's frame bodies (commands in between are handled here); the
        frames of one message together stay within max_msg_size"""
        frames, total = [], 0
        while True:
            flags, body = self.read_frame(self.max_msg_size - total)
            if flags & COMMAND:
                name, data = parse_command(body)
                if name == b"PING" and len(data) >= 2:  # TTL (2 bytes) + context
                    self.send(encode_command(b"PONG", data[2:]))
                continue
            frames.append(body)
            total += len(body)
            if not flags & MORE:
                return frames


def get_local_ip():
    """the IPv4 address of the default route's interface -- what the reference advertises
    for a service started with host=None (reth_buffer/reth_buffer/utils/__init__.py:29-32,
    netifaces' default gateway NIC); netifaces is absent, so the route comes from
    /proc/net/route and the address from SIOCGIFADDR.  Falls back to the source address of
    a (never sent) UDP datagram's route, then to the host name's address."""
    nic = None
    try:
        with open("/proc/net/route") as f:
            for line in f.readlines()[1:]:
                p = line.split()
                if len(p) > 7 and p[1] == "00000000" and int(p[3], 16) & 2 and p[7] == "00000000":
                    nic = p[0]
                    break
    except OSError:
        pass
    s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    try:
        if nic is not None:
            try:  # SIOCGIFADDR
                return socket.inet_ntoa(fcntl.ioctl(s.fileno(), 0x8915, struct.pack("256s", nic.encode()[:15]))[20:24])
            except OSError:
                pass
        try:
            s.connect(("192.0.2.1", 9))  # TEST-NET-1: connect() on UDP only picks the route
            ip = s.getsockname()[0]
            if ip and not ip.startswith("0."):
                return ip
        except OSError:
            pass
    finally:
        s.close()
    try:
        return socket.gethostbyname(socket.gethostname())
    except OSError:
        return "127.0.0.1"


class Peer:
    """a connecting ZMTP socket (b"PUSH" or b"REQ"): the reference Client's sockets
    (client.py:13-19, utils/__init__.py:51-59) for host processes without pyzmq"""

    def __init__(self, socket_type, addr, timeout=30.0):
        if not addr.startswith("tcp://"):
            raise ValueError(f"{addr!r}: only tcp:// endpoints")
        host, port = addr[len("tcp://"):].rsplit(":", 1)
        s = socket.create_connection((host, int(port)), timeout=timeout)
        s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        self.conn = Connection(s, socket_type)
        self.conn.handshake()

    def send(self, frames):
        self.conn.send(encode_message([frames] if isinstance(frames, (bytes, bytearray, memoryview)) else frames))

    def request(self, frames):
        """REQ: the empty delimiter, the request, then the reply's body frames"""
        self.send([b""] + list([frames] if isinstance(frames, (bytes, bytearray, memoryview)) else frames))
        reply = self.conn.read_message()
        cut = reply.index(b"") + 1 if b"" in reply else 0
        return reply[cut:]

    def close(self):
        try:
            self.conn.sock.close()
        except OSError:
            pass


class Endpoint:
    """a bound TCP listener serving ZMTP peers of one socket type (b"PULL" or b"REP")"""

    def __init__(self, socket_type, handler, host="127.0.0.1", port=0, max_msg_size=None):
        if socket_type not in (b"PULL", b"REP"):
            raise ValueError("socket_type: b'PULL' or b'REP'")
        self.socket_type = socket_type
        self.handler = handler
        self.max_msg_size = max_msg_size
        self._ls = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        self._ls.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        self._ls.bind((host, int(port)))
        self._ls.listen(64)
        self.host, self.port = self._ls.getsockname()[:2]
        self.errors = []  # handshake / protocol failures, for inspection
        self._conns = []
        self._closed = False
        self._thread = threading.Thread(target=self._accept_loop, daemon=True, name=f"zmtp-{socket_type.decode()}")
        self._thread.start()

    def addr(self, advertise=None):
        return f"tcp://{advertise or self.host}:{self.port}"

    def _accept_loop(self):
        while not self._closed:
            try:
                s, _ = self._ls.accept()
            except OSError:
                return
            s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            c = Connection(s, self.socket_type, self.max_msg_size)
            self._conns.append(c)
            threading.Thread(target=self._serve, args=(c,), daemon=True).start()

    def _serve(self, c):
        try:
            c.handshake()
            while not self._closed:
                frames = c.read_message()
                if self.socket_type == b"PULL":
                    self.handler(frames)
                else:  # REP: envelope = the frames up to and including the empty delimiter
                    cut = frames.index(b"") + 1 if b"" in frames else 0
                    reply = self.handler(frames[cut:])
                    c.send(encode_message(frames[:cut] + list(reply)))
        except (ConnectionError, OSError):
            pass
        except ZmtpError as e:
            self.errors.append(str(e))
        except Exception as e:  # a failing handler (or anything else) ends this connection only
            self.errors.append(f"{type(e).__name__}: {e}")
        finally:
            try:
                c.sock.close()
            except OSError:
                pass

    def close(self):
        self._closed = True
        try:
            self._ls.close()
        except OSError:
            pass
        for c in self._conns:
            try:
                c.sock.shutdown(socket.SHUT_RDWR)
            except OSError:
                pass
            try:
                c.sock.close()
            except OSError:
                pass
