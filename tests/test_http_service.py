"""HTTP/1.1 listener of the service layer (vsvc_http_start), on CPU.

The reference serves rag/vector-service's routes with net/http
(main.go:70-77) and retrieval-service posts to them with http.Post
(retrieval-service/main.go:229-233). These tests run the real listener and
handler code (csrc/service/*.cpp) over real sockets, with the CPU test double
of the engine C-ABI (tests/tsan/fake_engine.cpp, test-only: the product
engine has no CPU path), and check that the transport is transparent: every
HTTP answer equals what vsvc_handle answers in-process for the same request,
plus the net/http framing behaviours a Go client relies on (keep-alive,
pipelining, chunked bodies, Expect: 100-continue, HEAD, error statuses).
The GPU run of the same listener over the HIP engine is
tests/test_service_gpu.py::test_http_listener_gpu.
"""
import ctypes
import http.client
import json
import os
import socket
import subprocess
import threading
import time

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SVC = os.path.join(ROOT, "gorilla-rag---agentic-rag-with-mcp-using-golang-microservices_amd",
                   "csrc", "service")
SOURCES = [os.path.join(SVC, f) for f in ("json.cpp", "vector_service.cpp", "batcher.cpp",
                                          "loadgen.cpp", "http.cpp")]
FAKE = os.path.join(ROOT, "tests", "tsan", "fake_engine.cpp")
DIM = 16
CONFIG = {"collections": [{"name": "docs", "dim": DIM, "metric": "Cosine", "dtype": "f32"},
                          {"name": "kyc", "dim": DIM, "metric": "Dot", "dtype": "f32"}],
          "batching": {"enabled": True, "max_batch": 64}}


class _Lib:
    def __init__(self, path):
        L = ctypes.CDLL(path)
        vp, cp, sz = ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t
        L.vs_open.argtypes = [vp, ctypes.POINTER(vp)]
        L.vs_close.argtypes = [vp]
        L.vsvc_open.argtypes = [vp, cp, ctypes.POINTER(vp)]
        L.vsvc_close.argtypes = [vp]
        L.vsvc_handle.argtypes = [vp, cp, cp, cp, sz, ctypes.POINTER(ctypes.c_int),
                                  ctypes.POINTER(vp), ctypes.POINTER(sz), ctypes.POINTER(cp)]
        L.vsvc_free.argtypes = [vp]
        L.vsvc_http_start.argtypes = [vp, cp, ctypes.POINTER(vp)]
        L.vsvc_http_port.argtypes = [vp]
        L.vsvc_http_stop.argtypes = [vp]
        L.vsvc_loadgen.argtypes = [vp, cp, ctypes.POINTER(vp)]
        L.vsvc_stats.argtypes = [vp, ctypes.POINTER(vp)]
        L.vs_collection_placement.argtypes = [vp, cp, ctypes.POINTER(ctypes.c_int32)]
        self.L = L
        self.eng = vp()
        assert L.vs_open(None, ctypes.byref(self.eng)) == 0
        self.svc = vp()
        assert L.vsvc_open(self.eng, json.dumps(CONFIG).encode(), ctypes.byref(self.svc)) == 0

    def handle(self, method, path, body=b""):
        st, out, n, ct = ctypes.c_int(), ctypes.c_void_p(), ctypes.c_size_t(), ctypes.c_char_p()
        assert self.L.vsvc_handle(self.svc, method.encode(), path.encode(), body, len(body),
                                  ctypes.byref(st), ctypes.byref(out), ctypes.byref(n),
                                  ctypes.byref(ct)) == 0
        data = ctypes.string_at(out.value, n.value)
        self.L.vsvc_free(out)
        return st.value, data, ct.value.decode()

    def stats(self):
        out = ctypes.c_void_p()
        assert self.L.vsvc_stats(self.svc, ctypes.byref(out)) == 0
        d = json.loads(ctypes.string_at(out.value))
        self.L.vsvc_free(out)
        return d

    def serve(self, addr=b"127.0.0.1:0"):
        h = ctypes.c_void_p()
        rc = self.L.vsvc_http_start(self.svc, addr, ctypes.byref(h))
        return rc, h

    def loadgen(self, spec, svc=True):
        out = ctypes.c_void_p()
        rc = self.L.vsvc_loadgen(self.svc if svc else None, json.dumps(spec).encode(),
                                 ctypes.byref(out))
        rep = json.loads(ctypes.string_at(out.value)) if rc == 0 else None
        if out.value:
            self.L.vsvc_free(out)
        return rc, rep


@pytest.fixture(scope="module")
def lib(tmp_path_factory):
    d = tmp_path_factory.mktemp("httpsvc")
    so = str(d / "libvsvc_fake.so")
    subprocess.run(["g++", "-std=c++17", "-O1", "-fPIC", "-shared", "-pthread", *SOURCES, FAKE,
                    "-o", so], check=True, capture_output=True, timeout=600)
    lb = _Lib(so)
    rng = np.random.default_rng(5)
    for coll in ("docs", "kyc"):
        pts = [{"id": f"{i:08x}-0000-4000-8000-{i:012x}",
                "vector": [float(x) for x in rng.standard_normal(DIM)],
                "payload": {"text": f"{coll} chunk {i}", "document_id": f"d{i % 7}",
                            "page": i % 11}} for i in range(300)]
        st, body, _ = lb.handle("POST", "/upsert",
                                json.dumps({"collection": coll, "points": pts}).encode())
        assert st == 200, body
    yield lb
    lb.L.vsvc_close(lb.svc)
    lb.L.vs_close(lb.eng)


@pytest.fixture()
def server(lib):
    rc, h = lib.serve()
    assert rc == 0
    port = lib.L.vsvc_http_port(h)
    assert 0 < port < 65536
    yield port
    lib.L.vsvc_http_stop(h)


def _search_body(seed, coll="docs", k=5):
    q = np.random.default_rng(seed).standard_normal(DIM)
    return json.dumps({"collection": coll, "filter": None, "query": [float(x) for x in q],
                       "top_k": k}).encode()


def _raw(port):
    s = socket.create_connection(("127.0.0.1", port), timeout=10)
    s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
    return s


def _read_response(s, buf=b"", head=False):
    """One HTTP/1.1 response (Content-Length framed; no body after a HEAD)
    from socket s; returns (status, headers, body, rest_of_buffer)."""
    while b"\r\n\r\n" not in buf:
        chunk = s.recv(65536)
        if not chunk:
            raise ConnectionError("closed before a response head")
        buf += chunk
    hd, buf = buf.split(b"\r\n\r\n", 1)
    lines = hd.decode().split("\r\n")
    status = int(lines[0].split(" ")[1])
    hdr = {}
    for ln in lines[1:]:
        k, v = ln.split(":", 1)
        hdr[k.strip().lower()] = v.strip()
    n = 0 if head else int(hdr.get("content-length", "0"))
    while len(buf) < n:
        chunk = s.recv(65536)
        if not chunk:
            raise ConnectionError("closed inside a body")
        buf += chunk
    return status, hdr, buf[:n], buf[n:]


def _closed(s):
    try:
        return s.recv(1) == b""
    except (ConnectionResetError, socket.timeout):
        return True


def test_answers_equal_in_process_handler(lib, server):
    c = http.client.HTTPConnection("127.0.0.1", server, timeout=10)
    cases = [("POST", "/search", _search_body(1)), ("POST", "/search", _search_body(2, "kyc", 9)),
             ("POST", "/search", _search_body(3, "docs", 0)),
             ("POST", "/search", b'{"collection":"nope","query":[1],"top_k":3}'),
             ("POST", "/search", b"{bad json"), ("GET", "/search", b""),
             ("GET", "/health", b""), ("GET", "/collections", b""), ("POST", "/collections", b""),
             ("GET", "/nope", b""), ("POST", "/upsert", b'{"collection":"docs","points":[{"id":1}]}')]
    for method, path, body in cases:
        c.request(method, path, body=body, headers={"Content-Type": "application/json"})
        r = c.getresponse()
        got = r.read()
        st, want, ct = lib.handle(method, path, body)
        assert (r.status, got) == (st, want), (method, path, r.status, got[:200], want[:200])
        assert r.getheader("Content-Type") == ct
        assert r.getheader("Content-Length") == str(len(want))
        assert r.getheader("Date", "").endswith(" GMT")
        if ct.startswith("text/plain"):  # http.Error
            assert r.getheader("X-Content-Type-Options") == "nosniff"
    c.close()
    # a search reply is the reference's shape
    st, body, _ = lib.handle("POST", "/search", _search_body(1))
    doc = json.loads(body)
    assert set(doc) == {"results", "count"} and doc["count"] == 5
    assert {"id", "score", "payload"} <= set(doc["results"][0])


def test_keep_alive_and_query_string(lib, server):
    c = http.client.HTTPConnection("127.0.0.1", server, timeout=10)
    c.connect()
    sock = c.sock
    for i in range(20):
        c.request("POST", "/search?trace=1&x=%d" % i, body=_search_body(10 + i))
        r = c.getresponse()
        assert r.status == 200
        assert r.read() == lib.handle("POST", "/search", _search_body(10 + i))[1]
        assert c.sock is sock  # one connection for all of them
    c.close()


def test_pipelined_requests_answered_in_order(lib, server):
    s = _raw(server)
    bodies = [_search_body(40 + i, "kyc" if i % 2 else "docs", 3 + i) for i in range(6)]
    req = b"".join(b"POST /search HTTP/1.1\r\nHost: x\r\nContent-Length: %d\r\n\r\n%s"
                   % (len(b), b) for b in bodies)
    req += b"GET /health HTTP/1.1\r\nHost: x\r\n\r\n"
    s.sendall(req)
    rest = b""
    for b in bodies:
        st, hdr, body, rest = _read_response(s, rest)
        assert st == 200 and body == lib.handle("POST", "/search", b)[1]
    st, hdr, body, rest = _read_response(s, rest)
    assert st == 200 and json.loads(body)["status"] == "healthy"
    s.close()


def test_chunked_body_and_expect_continue(lib, server):
    body = _search_body(77, "docs", 7)
    want = lib.handle("POST", "/search", body)[1]
    # chunked, with a chunk extension and a trailer
    s = _raw(server)
    parts = [body[:10], body[10:300], body[300:]]
    enc = b"".join(b"%x;ext=1\r\n%s\r\n" % (len(p), p) for p in parts) + b"0\r\nX-T: 1\r\n\r\n"
    s.sendall(b"POST /search HTTP/1.1\r\nHost: x\r\nTransfer-Encoding: chunked\r\n\r\n" + enc)
    st, hdr, got, _ = _read_response(s)
    assert st == 200 and got == want
    # Expect: 100-continue: the interim response comes before the body is sent
    s.sendall(b"POST /search HTTP/1.1\r\nHost: x\r\nExpect: 100-continue\r\n"
              b"Content-Length: %d\r\n\r\n" % len(body))
    st, hdr, got, rest = _read_response(s)
    assert st == 100 and got == b""
    s.sendall(body)
    st, hdr, got, _ = _read_response(s, rest)
    assert st == 200 and got == want
    s.close()


def test_chunked_body_in_pieces(lib, server):
    """Many small chunks arriving in separate segments: the framing resumes
    where it stopped (csrc/service/http.cpp ChunkScan) and decodes exactly."""
    body = _search_body(91, "kyc", 12)
    want = lib.handle("POST", "/search", body)[1]
    enc = b"".join(b"%x\r\n%s\r\n" % (len(body[i:i + 7]), body[i:i + 7])
                   for i in range(0, len(body), 7)) + b"0\r\n\r\n"
    s = _raw(server)
    s.sendall(b"POST /search HTTP/1.1\r\nHost: x\r\nTransfer-Encoding: chunked\r\n\r\n")
    for i in range(0, len(enc), 1000):
        s.sendall(enc[i:i + 1000])
        time.sleep(0.002)
    st, hdr, got, _ = _read_response(s)
    assert st == 200 and got == want
    s.close()


def test_head_and_connection_close(lib, server):
    s = _raw(server)
    s.sendall(b"HEAD /health HTTP/1.1\r\nHost: x\r\n\r\n")
    st, hdr, body, rest = _read_response(s, head=True)
    # HEAD: the GET answer's headers and no body bytes
    _, full, _ = lib.handle("GET", "/health")
    assert st == 200 and int(hdr["content-length"]) == len(full)
    s.settimeout(0.3)
    try:
        assert s.recv(1) == b""  # nothing more than the head ...
        pytest.fail("connection closed after HEAD")
    except socket.timeout:
        pass  # ... and the connection stays open
    s.settimeout(10)
    s.sendall(b"GET /collections HTTP/1.1\r\nHost: x\r\nConnection: close\r\n\r\n")
    st, hdr, body, rest = _read_response(s, rest)
    assert st == 200 and hdr.get("connection") == "close"
    assert _closed(s)
    s.close()
    # HTTP/1.0 without keep-alive: one request per connection
    s = _raw(server)
    s.sendall(b"GET /health HTTP/1.0\r\n\r\n")
    st, hdr, body, _ = _read_response(s)
    assert st == 200 and _closed(s)
    s.close()
    # HTTP/1.0 with keep-alive: echoed, and the connection serves a second request
    s = _raw(server)
    s.sendall(b"GET /health HTTP/1.0\r\nConnection: keep-alive\r\n\r\n")
    st, hdr, body, rest = _read_response(s)
    assert st == 200 and hdr.get("connection") == "keep-alive"
    s.sendall(b"GET /collections HTTP/1.0\r\n\r\n")
    st, hdr, body, _ = _read_response(s, rest)
    assert st == 200 and _closed(s)
    s.close()


@pytest.mark.parametrize("req,status", [
    (b"GARBAGE\r\n\r\n", 400),
    (b"GET /health HTTP/1.1\r\n\r\n", 400),                        # no Host
    (b"GET /health HTTP/2.0\r\nHost: x\r\n\r\n", 505),
    (b"POST /search HTTP/1.1\r\nHost: x\r\nTransfer-Encoding: gzip\r\n\r\n", 501),
    (b"POST /search HTTP/1.1\r\nHost: x\r\nContent-Length: 3\r\nContent-Length: 4\r\n\r\nabcd", 400),
    (b"POST /search HTTP/1.1\r\nHost: x\r\nContent-Length: -1\r\n\r\n", 400),
    (b"POST /search HTTP/1.1\r\nHost: x\r\nExpect: magic\r\n\r\n", 417),
    (b"POST /search HTTP/1.1\r\nHost: x\r\nTransfer-Encoding: chunked\r\n\r\nzz\r\n", 400),
    (b"GET /health HTTP/1.1\r\nHost: x\r\n folded: y\r\n\r\n", 400),
    # two Transfer-Encoding lines: ambiguous framing (net/http: "too many
    # transfer encodings"), even when both say chunked
    (b"POST /search HTTP/1.1\r\nHost: x\r\nTransfer-Encoding: chunked\r\n"
     b"Transfer-Encoding: chunked\r\n\r\n0\r\n\r\n", 501),
    (b"POST /search HTTP/1.1\r\nHost: x\r\nTransfer-Encoding: gzip, chunked\r\n\r\n", 501),
    # a body announced past the 256 MiB request cap
    (b"POST /upsert HTTP/1.1\r\nHost: x\r\nContent-Length: 268435457\r\n\r\n", 413),
])
def test_malformed_requests(server, req, status):
    s = _raw(server)
    s.sendall(req)
    st, hdr, body, _ = _read_response(s)
    assert st == status, body
    assert hdr.get("connection") == "close" and _closed(s)
    s.close()


def test_oversized_head_is_431(server):
    s = _raw(server)
    s.sendall(b"GET /health HTTP/1.1\r\nHost: x\r\nX-Big: " + b"a" * (1 << 20) + b"\r\n")
    st, hdr, body, _ = _read_response(s)
    assert st == 431
    s.close()


def test_chunked_trailer_is_bounded(server):
    """Trailer lines count against the 1 MiB header limit: an endless trailer
    is refused (400) instead of growing the buffer (and is framed line by
    line, not rescanned from the last chunk on every receive)."""
    s = _raw(server)
    s.sendall(b"POST /search HTTP/1.1\r\nHost: x\r\nTransfer-Encoding: chunked\r\n\r\n"
              b"2\r\n{}\r\n0\r\n")
    line = b"X-T: " + b"a" * 4000 + b"\r\n"
    try:
        for _ in range(300):  # ~1.2 MB of trailer lines
            s.sendall(line * 1)
    except (BrokenPipeError, ConnectionResetError):
        pass
    st, hdr, body, _ = _read_response(s)
    assert st == 400 and _closed(s)
    s.close()


def test_chunked_body_past_cap_is_refused(server):
    s = _raw(server)
    s.sendall(b"POST /upsert HTTP/1.1\r\nHost: x\r\nTransfer-Encoding: chunked\r\n\r\n"
              b"10000001\r\n")  # one chunk of 256 MiB + 1
    st, hdr, body, _ = _read_response(s)
    assert st == 400 and _closed(s)
    s.close()


def test_concurrent_clients(lib, server):
    errors = []

    def client(t):
        try:
            c = http.client.HTTPConnection("127.0.0.1", server, timeout=30)
            for i in range(15):
                b = _search_body(1000 * t + i, "kyc" if (t + i) % 3 == 0 else "docs", 1 + (i % 20))
                c.request("POST", "/search", body=b)
                r = c.getresponse()
                got = r.read()
                if r.status != 200 or got != lib.handle("POST", "/search", b)[1]:
                    errors.append((t, i, r.status))
            c.close()
        except Exception as e:  # noqa: BLE001
            errors.append((t, repr(e)))

    th = [threading.Thread(target=client, args=(t,)) for t in range(16)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors, errors[:5]


def test_loadgen_over_http(lib, server):
    for keepalive in (True, False):
        rc, rep = lib.loadgen({"collections": ["docs", "kyc"], "dim": DIM, "clients": 8,
                               "seconds": 0.4, "k_min": 3, "k_max": 50,
                               "http": "127.0.0.1:%d" % server, "keepalive": keepalive},
                              svc=False)
        assert rc == 0
        assert rep["transport"] == "http"
        assert rep["errors"] == 0, rep["first_error"]
        assert rep["requests"] > 0 and rep["qps"] > 0
    rc, rep = lib.loadgen({"collections": ["docs"], "dim": DIM, "clients": 2, "seconds": 0.2})
    assert rc == 0 and rep["transport"] == "inproc" and rep["errors"] == 0
    # bad address / nothing listening
    assert lib.loadgen({"collections": ["docs"], "dim": DIM, "http": "nope"})[0] == -1
    rc, rep = lib.loadgen({"collections": ["docs"], "dim": DIM, "clients": 1, "seconds": 0.1,
                           "http": "127.0.0.1:1"}, svc=False)
    assert rc == 0 and rep["errors"] == rep["requests"] > 0
    assert rep["first_error"].startswith("transport:")


def test_bad_address_and_stop_with_idle_connections(lib):
    assert lib.serve(b"not-an-address")[0] == -1
    assert lib.serve(b"10.255.255.255.1:80")[0] == -1
    rc, h = lib.serve()
    assert rc == 0
    port = lib.L.vsvc_http_port(h)
    idle = [_raw(port) for _ in range(8)]
    c = http.client.HTTPConnection("127.0.0.1", port, timeout=10)
    c.request("GET", "/health")
    assert c.getresponse().status == 200
    t0 = time.time()
    lib.L.vsvc_http_stop(h)
    assert time.time() - t0 < 5.0
    for s in idle:
        assert _closed(s)
        s.close()
    with pytest.raises(OSError):
        socket.create_connection(("127.0.0.1", port), timeout=2).recv(1)


def test_batcher_policies_over_http(lib, server):
    """The batcher seen through the listener (csrc/service/batcher.h): a lone
    request on an idle batcher runs as its own engine call (caller_runs);
    concurrent keep-alive clients are coalesced into multi-query calls, two
    in flight, each request still answered with exactly its own top k."""
    st0 = lib.stats()
    # two workers per device the collections live on (the test double
    # pretends two devices, vs_collection_placement by name hash)
    devs = set()
    for coll in json.loads(lib.handle("GET", "/collections")[1])["collections"]:
        d = ctypes.c_int32()
        assert lib.L.vs_collection_placement(lib.eng, coll.encode(), ctypes.byref(d)) == 0
        devs.add(d.value)
    assert st0["batching"]["workers"] == 2 * len(devs) and st0["batching"]["caller_runs"]
    c = http.client.HTTPConnection("127.0.0.1", server, timeout=30)
    for i in range(10):
        b = _search_body(5000 + i, "docs", 4)
        c.request("POST", "/search", body=b)
        r = c.getresponse()
        assert r.status == 200 and r.read() == lib.handle("POST", "/search", b)[1]
    c.close()
    st1 = lib.stats()
    # each sequential request (and each in-process check after it) was alone
    assert st1["requests"] - st0["requests"] == 20
    assert st1["engine_calls"] - st0["engine_calls"] == 20
    rc, rep = lib.loadgen({"collections": ["docs", "kyc"], "dim": DIM, "clients": 32,
                           "seconds": 0.6, "k_min": 1, "k_max": 60,
                           "http": "127.0.0.1:%d" % server}, svc=False)
    assert rc == 0 and rep["errors"] == 0, rep
    st2 = lib.stats()
    calls = st2["engine_calls"] - st1["engine_calls"]
    reqs = st2["requests"] - st1["requests"]
    assert reqs == rep["requests"] and calls < reqs and st2["largest_call"] >= 2, (st2, rep)
