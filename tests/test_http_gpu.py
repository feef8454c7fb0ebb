"""/search over real HTTP on the device: the listener
(vsvc_http_start) in front of the handler mirror and the HIP engine, driven
the way retrieval-service drives vector-service (http.Post of
{"collection","filter","query","top_k"}, rag/retrieval-service/main.go:
219-276), every reply checked against the oracle; and the vector-service
process itself (lib/vsearch_server: PORT, VS_SERVICE_CONFIG, VS_BULK,
VS_DATA_DIR), restarted over its own snapshot."""
import http.client
import json
import os
import signal
import subprocess
import threading
import uuid

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SERVER = os.path.join(ROOT, "gorilla-rag---agentic-rag-with-mcp-using-golang-microservices_amd",
                      "lib", "vsearch_server")
CFG = {"collections": [{"name": "b16", "dim": 768, "metric": "Cosine", "dtype": "bf16"},
                       {"name": "f32", "dim": 768, "metric": "Cosine", "dtype": "f32"}],
       "batching": {"max_wait_us": 20000}}


@pytest.fixture(scope="module")
def svcmod(pkg):
    from importlib import import_module
    return import_module(pkg.__name__ + ".service")


def _ids(n, seed):
    rng = np.random.default_rng(seed)
    return [str(uuid.UUID(bytes=rng.bytes(16), version=4)) for _ in range(n)]


def _fill(s, orc, coll, n, seed, bf16):
    X = orc.generate(seed, 0, n, 768)
    ids = _ids(n, seed)
    for lo in range(0, n, 512):
        st, body, _ = s.handle("POST", "/upsert", json.dumps({"collection": coll, "points": [
            {"id": ids[i], "vector": X[i].tolist(), "payload": {"i": i, "text": f"chunk {i}"}}
            for i in range(lo, min(n, lo + 512))]}).encode())
        assert st == 200, body
    return orc.preprocess(X, True, bf16), ids


def _check_reply(orc, body, Xp, row_of, q, k, bf16):
    res = json.loads(body)
    assert res["count"] == len(res["results"]) == min(k, Xp.shape[0])
    rows = np.array([[row_of(r["id"]) for r in res["results"]]], np.uint64)
    scores = np.array([[r["score"] for r in res["results"]]])
    qp = orc.preprocess(q[None, :], True, bf16)
    s32, s64, rr, cc = orc.search(Xp, qp, k)
    resc = orc.rescore(Xp, qp, rows, np.array([k], np.uint32))
    bad = orc.check_topk(scores, rows, np.array([k]), s64, rr, cc, resc, 1e-5)
    assert not bad, bad[:3]
    return res


def test_http_listener_gpu(pkg, svcmod, orc):
    """48 concurrent HTTP clients (one request each, released together) over
    two collections with k in [3, 50]: exact replies, coalesced by the
    batcher; then the closed-loop load generator over TCP."""
    eng = pkg.VectorEngine(device=0)
    s = svcmod.VectorService(eng, CFG)
    try:
        data = {"b16": _fill(s, orc, "b16", 4000, 61, True),
                "f32": _fill(s, orc, "f32", 3000, 62, False)}
        with s.serve("127.0.0.1:0") as lis:
            nreq = 48
            Q = orc.generate(orc.SEED_QUERY, 900, nreq, 768)
            ks = [3 + (11 * i) % 48 for i in range(nreq)]
            colls = ["b16" if i % 3 else "f32" for i in range(nreq)]
            conns = [http.client.HTTPConnection("127.0.0.1", lis.port, timeout=60)
                     for _ in range(nreq)]
            for c in conns:
                c.connect()
            replies = [None] * nreq
            gate = threading.Barrier(nreq)

            def client(i):
                body = json.dumps({"collection": colls[i], "filter": None,
                                   "query": Q[i].tolist(), "top_k": ks[i]})
                gate.wait()
                conns[i].request("POST", "/search", body=body,
                                 headers={"Content-Type": "application/json"})
                r = conns[i].getresponse()
                replies[i] = (r.status, r.getheader("Content-Type"), r.read())

            th = [threading.Thread(target=client, args=(i,)) for i in range(nreq)]
            for t in th:
                t.start()
            for t in th:
                t.join()
            for c in conns:
                c.close()
            for i in range(nreq):
                st, ct, body = replies[i]
                assert st == 200 and ct == "application/json", body[:200]
                Xp, ids = data[colls[i]]
                pos = {u: j for j, u in enumerate(ids)}
                res = _check_reply(orc, body, Xp, pos.__getitem__, Q[i], ks[i], colls[i] == "b16")
                assert res["results"][0]["payload"]["text"] == \
                    "chunk %d" % res["results"][0]["payload"]["i"]
            st = s.stats()
            assert st["requests"] >= nreq and st["engine_calls"] < st["requests"], st
            # closed loop over TCP, keep-alive and one connection per request
            for ka in (True, False):
                rep = s.loadgen(["b16", "f32"], 768, clients=24, seconds=1.0, k_min=3, k_max=50,
                                http="127.0.0.1:%d" % lis.port, keepalive=ka)
                assert rep["transport"] == "http"
                assert rep["errors"] == 0, rep["first_error"]
                assert rep["requests"] > 50, rep
    finally:
        s.close()
        eng.close()


def test_c1_over_http(pkg, svcmod, orc):
    """Config C1 end to end over HTTP with the reference's defaults (3 x 768
    Cosine fp32 collections): ingest-service's /upsert bodies (2 documents x
    110 chunks + 1, payload text / document_id / position) posted to the
    listener, then retrieval-service's /search bodies (top_k 5, and top_k 0
    -> 5) checked against the oracle; every HTTP reply equals the in-process
    handler's bytes."""
    eng = pkg.VectorEngine(device=0)
    s = svcmod.VectorService(eng)
    try:
        n, dim = 221, 768
        X = orc.generate(4040, 0, n, dim) * 3.0  # not unit: the upsert normalises
        ids = _ids(n, 4040)
        docs = [(0, 110, "doc-a"), (110, 220, "doc-b"), (220, 221, "test_doc")]
        with s.serve("127.0.0.1:0") as lis:
            c = http.client.HTTPConnection("127.0.0.1", lis.port, timeout=60)
            for lo, hi, doc in docs:
                body = json.dumps({"collection": "regulatory_docs", "points": [
                    {"id": ids[i], "vector": [float(x) for x in X[i]],
                     "payload": {"text": f"chunk {i} of {doc}", "document_id": doc,
                                 "position": i - lo}} for i in range(lo, hi)]})
                c.request("POST", "/upsert", body=body,
                          headers={"Content-Type": "application/json"})
                r = c.getresponse()
                out = json.loads(r.read())
                assert r.status == 200 and out == {"collection": "regulatory_docs",
                                                   "points": hi - lo, "status": "success"}
            Xp = orc.preprocess(X, True, False)
            pos = {u: j for j, u in enumerate(ids)}
            Q = orc.generate(orc.SEED_QUERY, 4041, 6, dim)
            for i in range(6):
                top_k = 0 if i == 5 else 5
                body = json.dumps({"collection": "regulatory_docs", "filter": None,
                                   "query": [float(x) for x in Q[i]], "top_k": top_k})
                c.request("POST", "/search", body=body,
                          headers={"Content-Type": "application/json"})
                r = c.getresponse()
                got = r.read()
                assert r.status == 200
                res = _check_reply(orc, got, Xp, pos.__getitem__, Q[i], 5, False)
                for hit in res["results"]:
                    j = pos[hit["id"]]
                    doc = "doc-a" if j < 110 else ("doc-b" if j < 220 else "test_doc")
                    assert hit["payload"]["document_id"] == doc
                assert got == s.handle("POST", "/search", body.encode())[1]
            c.close()
    finally:
        s.close()
        eng.close()


def _bulk_row(uid):
    g = uid.split("-")
    return ((int(g[3], 16) << 48) | int(g[4], 16)) & ((1 << 62) - 1)


def _start_server(env):
    p = subprocess.Popen([SERVER], env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                         text=True)
    seen = []
    for _ in range(50):  # RCCL prints its version line first in the multi-device mode
        line = p.stdout.readline()
        seen.append(line)
        if "starting on port" in line or not line:
            break
    if "starting on port" not in line:
        p.kill()
        raise AssertionError("server did not start: %r %s" % (seen, p.stderr.read()[-2000:]))
    return p, int(line.split()[-1])


def _post(port, body):
    c = http.client.HTTPConnection("127.0.0.1", port, timeout=60)
    c.request("POST", "/search", body=json.dumps(body), headers={"Content-Type": "application/json"})
    r = c.getresponse()
    out = (r.status, r.read())
    c.close()
    return out


def test_vsearch_server_sharded(tmp_path, orc):
    """VS_DEVICES=0,0: the server's multi-device mode (vs_open_multi, two
    row-striped shards, here both on the box's one GPU, RCCL with a
    1-device communicator) answers /search exactly like one device."""
    assert os.path.exists(SERVER), "run __graft_entry__.build()"
    cfgp = tmp_path / "cfg.json"
    cfgp.write_text(json.dumps({"collections": [
        {"name": "kyc_docs", "dim": 768, "metric": "Cosine", "dtype": "bf16"}]}))
    n, seed = 30001, 99
    env = dict(os.environ, PORT="0", VS_SERVICE_CONFIG=str(cfgp), VS_DEVICES="0,0",
               VS_BULK="kyc_docs=%d:%d" % (n, seed))
    env.pop("VS_DATA_DIR", None)
    X = orc.generate(seed, 0, n, 768, bf16=True)
    Q = orc.generate(orc.SEED_QUERY, 501, 3, 768)
    p, port = _start_server(env)
    try:
        for i in range(3):
            for k in (1, 10, 50):
                st, body = _post(port, {"collection": "kyc_docs", "query": Q[i].tolist(),
                                        "top_k": k, "filter": None})
                assert st == 200, body
                _check_reply(orc, body, X, _bulk_row, Q[i], k, True)
        c = http.client.HTTPConnection("127.0.0.1", port, timeout=30)
        c.request("GET", "/health")
        r = c.getresponse()
        assert r.status == 200 and json.loads(r.read())["status"] == "healthy"
        c.close()
    finally:
        p.send_signal(signal.SIGTERM)
        out, err = p.communicate(timeout=120)
    assert p.returncode == 0, err[-2000:]


def test_vsearch_server_process(tmp_path, orc):
    """lib/vsearch_server as the vector-service process: bulk rows from
    VS_BULK, /search over HTTP checked against the oracle, SIGTERM writes the
    snapshot to VS_DATA_DIR, and a restarted server answers the same bytes."""
    assert os.path.exists(SERVER), "run __graft_entry__.build()"
    cfgp = tmp_path / "cfg.json"
    cfgp.write_text(json.dumps({"collections": [
        {"name": "regulatory_docs", "dim": 768, "metric": "Cosine", "dtype": "bf16"}]}))
    data = tmp_path / "data"
    n, seed = 20000, 4242
    env = dict(os.environ, PORT="0", VS_SERVICE_CONFIG=str(cfgp), VS_DATA_DIR=str(data),
               VS_BULK="regulatory_docs=%d:%d" % (n, seed))
    X = orc.generate(seed, 0, n, 768, bf16=True)
    Q = orc.generate(orc.SEED_QUERY, 77, 4, 768)
    p, port = _start_server(env)
    try:
        c = http.client.HTTPConnection("127.0.0.1", port, timeout=30)
        c.request("GET", "/health")
        r = c.getresponse()
        assert r.status == 200 and json.loads(r.read())["status"] == "healthy"
        c.close()
        first = []
        for i in range(4):
            st, body = _post(port, {"collection": "regulatory_docs", "query": Q[i].tolist(),
                                    "top_k": 10, "filter": None})
            assert st == 200, body
            _check_reply(orc, body, X, _bulk_row, Q[i], 10, True)
            first.append(body)
        st, body = _post(port, {"collection": "nope", "query": Q[0].tolist(), "top_k": 3})
        assert st == 500 and b"Search failed" in body
    finally:
        p.send_signal(signal.SIGTERM)
        out, err = p.communicate(timeout=120)
    assert p.returncode == 0, err[-2000:]
    assert (data / "regulatory_docs.vsnap").exists()
    env.pop("VS_BULK")
    p, port = _start_server(env)
    try:
        for i in range(4):
            st, body = _post(port, {"collection": "regulatory_docs", "query": Q[i].tolist(),
                                    "top_k": 10, "filter": None})
            assert st == 200 and body == first[i]
    finally:
        p.send_signal(signal.SIGTERM)
        p.communicate(timeout=120)
    assert p.returncode == 0
