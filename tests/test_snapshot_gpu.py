"""Snapshot / restore of resident collections on the device.

The device checksum (vs_checksum, HIP streaming reduction) is checked bit for
bit against the oracle's sequential restatement; snapshot -> restore round
trips are bit-exact and give identical search results; corrupt, truncated or
foreign files are refused without leaving a collection behind.
"""
import json
import os
import struct

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HDR = struct.Struct("<8sIIIiiIQQQQQ56s")  # vs_engine.cpp SnapHeader (128 bytes)


def _stored_bytes(eng, name):
    """The collection's rows exactly as stored (bf16 = the upper half of the f32 upcast)."""
    info = eng.collection_info(name)
    x = eng.read_rows(name, 0, info["rows"])
    if info["dtype"] == 1:
        return (x.view(np.uint32) >> 16).astype("<u2").tobytes()
    return x.astype("<f4").tobytes()


@pytest.mark.parametrize("dtype", [0, 1])
@pytest.mark.parametrize("dim,n", [(768, 5000), (100, 777), (3, 5), (768, 0), (1, 1)])
def test_checksum_matches_oracle(engine, orc, dtype, dim, n):
    name = f"ck_{dtype}_{dim}_{n}"
    engine.create_collection(name, dim, 0, dtype)
    if n:
        engine.generate(name, n, orc.SEED_CORPUS)
    data = _stored_bytes(engine, name)
    assert len(data) == n * dim * (2 if dtype else 4)
    assert engine.checksum(name) == orc.checksum(data) == orc.np_checksum(data)
    engine.drop_collection(name)


@pytest.mark.parametrize("dtype", [0, 1])
def test_snapshot_restore_roundtrip(engine, orc, tmp_path, dtype, pkg):
    n, dim = 40_000, 768
    engine.create_collection("snap", dim, 0, dtype, 0, 1000)  # row_base 1000 travels too
    engine.generate("snap", n, orc.SEED_CORPUS)
    raw = orc.generate(3, 0, 50, dim) * 2.0
    engine.upsert("snap", np.arange(100, 150), raw)  # overwrite some rows
    path = str(tmp_path / "snap.vsnap")
    engine.snapshot("snap", path)
    blob = open(path, "rb").read()
    h = HDR.unpack(blob[:128])
    magic, ver, hb, d, metric, dt, elem, rows, rbase, nbytes, dsum, hsum, _ = h
    assert (magic, ver, hb, d, metric, dt, elem) == (b"VSNAP01\0", 1, 128, dim, 0, dtype,
                                                     2 if dtype else 4)
    assert (rows, rbase, nbytes) == (n, 1000, n * dim * elem) and len(blob) == 128 + nbytes
    assert dsum == engine.checksum("snap") == orc.checksum(blob[128:])
    assert blob[128:] == _stored_bytes(engine, "snap")
    # restore on this engine and on a fresh one: bit-exact rows, same answers
    engine.restore("snap2", path)
    eng2 = pkg.VectorEngine(device=0)
    try:
        eng2.restore("snap", path)
        for e, nm in ((engine, "snap2"), (eng2, "snap")):
            info = e.collection_info(nm)
            assert info["rows"] == n and info["dim"] == dim and info["dtype"] == dtype
            assert _stored_bytes(e, nm) == blob[128:]
        Q = orc.generate(orc.SEED_QUERY, 0, 64, dim)
        a = engine.search("snap", Q, 10)
        for e, nm in ((engine, "snap2"), (eng2, "snap")):
            b = e.search(nm, Q, 10)
            assert all(np.array_equal(x, y) for x, y in zip(a, b))
        assert a[1].min() >= 1000  # global rows carry row_base
    finally:
        eng2.close()
    engine.drop_collection("snap")
    engine.drop_collection("snap2")


def test_restore_refuses_bad_files(engine, orc, tmp_path, pkg):
    engine.create_collection("src", 64, 0, 1)
    engine.generate("src", 3000, orc.SEED_CORPUS)
    good = str(tmp_path / "good.vsnap")
    engine.snapshot("src", good)
    blob = bytearray(open(good, "rb").read())
    cases = {}
    flip = bytearray(blob)
    flip[128 + 5000] ^= 0x10  # one bit of the data
    cases["flip"] = flip
    cases["trunc"] = blob[:-7]
    hdr = bytearray(blob)
    hdr[16] ^= 1  # dim: header checksum no longer matches
    cases["header"] = hdr
    cases["magic"] = b"NOTASNAP" + blob[8:]
    for tag, data in cases.items():
        p = tmp_path / f"{tag}.vsnap"
        p.write_bytes(bytes(data))
        with pytest.raises(pkg.VSError) as ei:
            engine.restore("bad", str(p))
        assert ei.value.code == -8, (tag, ei.value)  # VS_ERR_IO
        with pytest.raises(pkg.VSError):
            engine.collection_info("bad")  # nothing left behind
    with pytest.raises(pkg.VSError) as ei:
        engine.restore("src", good)  # name taken
    assert ei.value.code == -6
    with pytest.raises(pkg.VSError) as ei:
        engine.restore("x", str(tmp_path / "missing.vsnap"))
    assert ei.value.code == -8
    engine.drop_collection("src")


def test_service_snapshot_restore(pkg, orc, tmp_path):
    """Whole vector-service state: bulk points, upserted points with payloads,
    an overwritten bulk point; the restored service answers byte-identically."""
    from importlib import import_module
    svcmod = import_module(pkg.__name__ + ".service")
    cfg = {"collections": [{"name": "docs", "dim": 768, "metric": "Cosine", "dtype": "bf16"},
                           {"name": "empty", "dim": 768}]}
    eng = pkg.VectorEngine(device=0)
    s = svcmod.VectorService(eng, cfg)
    s.bulk_generate("docs", 3000, orc.SEED_CORPUS)
    X = orc.generate(9, 0, 20, 768)
    ids = [f"00000000-0000-4000-8000-{i:012x}" for i in range(20)]
    pts = [{"id": ids[i], "vector": X[i].tolist(), "payload": {"text": f"t{i}", "document_id": "d"}}
           for i in range(20)]
    pts.append({"id": s.point_id("docs", 5), "vector": X[0].tolist(), "payload": {"over": 1}})
    st, body, _ = s.handle("POST", "/upsert", json.dumps({"collection": "docs", "points": pts}).encode())
    assert st == 200, body
    queries = [X[i].tolist() for i in range(0, 20, 4)] + \
        [orc.generate(orc.SEED_CORPUS, 0, 3000, 768, bf16=True)[77].tolist()]
    before = [s.handle("POST", "/search", json.dumps({"collection": "docs", "query": q,
                                                      "top_k": 7}).encode())[1] for q in queries]
    s.snapshot(str(tmp_path))
    assert sorted(os.listdir(tmp_path)) == ["docs.points.json", "docs.vsnap", "empty.points.json",
                                            "empty.vsnap"]
    s.close()
    eng.close()

    eng = pkg.VectorEngine(device=0)
    s = svcmod.VectorService(eng, cfg)
    try:
        s.restore(str(tmp_path))
        after = [s.handle("POST", "/search", json.dumps({"collection": "docs", "query": q,
                                                         "top_k": 7}).encode())[1] for q in queries]
        assert after == before
        assert s.point_id("docs", 3000 + 3) == ids[3]
        # the restored UUID map still routes overwrites by id
        st, _, _ = s.handle("POST", "/upsert", json.dumps({"collection": "docs", "points": [
            {"id": ids[3], "vector": (-X[3]).tolist()}]}).encode())
        assert st == 200 and eng.collection_info("docs")["rows"] == 3020
        with pytest.raises(pkg.VSError):
            s.restore(str(tmp_path))  # collections no longer empty
    finally:
        s.close()
        eng.close()


def test_search_runs_while_snapshot_writes(pkg, orc, tmp_path):
    """vs_snapshot holds only the collection's reader lock, never
    the engine's work lock, so searches (other collections and the same one)
    and /health complete while a large snapshot is being written."""
    import threading
    import time
    eng = pkg.VectorEngine(device=0)
    try:
        eng.create_collection("big", 768, 1, 1)
        eng.generate("big", 2_000_000, orc.SEED_CORPUS)  # 3.07 GB to write
        eng.create_collection("small", 768, 1, 1)
        eng.generate("small", 5000, orc.SEED_CORPUS)
        Q = orc.generate(orc.SEED_QUERY, 0, 4, 768)
        eng.search("small", Q, 10)  # warm
        done = threading.Event()
        err = []

        def snap():
            try:
                eng.snapshot("big", str(tmp_path / "big.vsnap"))
            except Exception as e:  # pragma: no cover - reported below
                err.append(e)
            finally:
                done.set()

        t = threading.Thread(target=snap)
        t.start()
        during = 0
        t0 = time.time()
        while not done.is_set() and time.time() - t0 < 60:
            eng.search("small", Q, 10)
            eng.search("big", Q[:1], 10)
            eng.health()
            if not done.is_set():
                during += 1
        t.join()
        assert not err, err
        assert during >= 1, "no search completed while the snapshot was being written"
        assert os.path.getsize(tmp_path / "big.vsnap") == 128 + 2_000_000 * 768 * 2
    finally:
        eng.close()


def _bulk_uuid(tag, r):
    """vector_service.cpp bulk_uuid: v4 UUID carrying the tag and the row."""
    hi, lo = (tag << 16) | 0x4000, (1 << 63) | r
    return (f"{hi >> 32:08x}-{(hi >> 16) & 0xFFFF:04x}-{hi & 0xFFFF:04x}-"
            f"{lo >> 48:04x}-{lo & 0xFFFFFFFFFFFF:012x}")


def _sidecar_service(pkg, svcmod, orc, d):
    cfg = {"collections": [{"name": "docs", "dim": 64, "dtype": "bf16"}]}
    eng = pkg.VectorEngine(device=0)
    s = svcmod.VectorService(eng, cfg)
    s.bulk_generate("docs", 100, orc.SEED_CORPUS)
    X = orc.generate(9, 0, 3, 64)
    pts = [{"id": f"00000000-0000-4000-8000-{i:012x}", "vector": X[i].tolist(),
            "payload": {"p": i}} for i in range(3)]
    pts.append({"id": s.point_id("docs", 7), "vector": X[0].tolist(), "payload": {"b": 1}})
    st, body, _ = s.handle("POST", "/upsert", json.dumps({"collection": "docs", "points": pts}).encode())
    assert st == 200, body
    s.snapshot(str(d))
    s.close()
    eng.close()


def test_service_restore_refuses_corrupt_sidecar(pkg, orc, tmp_path):
    """the whole sidecar is checked before the collection is
    touched; a malformed one leaves the service empty and usable."""
    from importlib import import_module
    svcmod = import_module(pkg.__name__ + ".service")
    _sidecar_service(pkg, svcmod, orc, tmp_path)
    good = json.loads((tmp_path / "docs.points.json").read_text())
    assert good["bulk"] == 100 and len(good["points"]) == 3 and good["bulk_payload"][0][0] == 7
    bad = {
        "bulk_fraction": dict(good, bulk=100.5),
        "bulk_negative": dict(good, bulk=-1),
        "payload_row_out_of_range": dict(good, bulk_payload=[[100, {"b": 1}]]),
        "payload_not_object": dict(good, bulk_payload=[[7, 3]]),
        "point_not_pair": dict(good, points=good["points"][:2] + [[good["points"][2][0]]]),
        "point_bad_uuid": dict(good, points=good["points"][:2] + [["zzz", {}]]),
        "point_duplicate": dict(good, points=good["points"][:2] + [good["points"][0]]),
        "point_is_bulk_id": dict(good, points=good["points"][:2] + [[_bulk_uuid(good["bulk_tag"], 5), {}]]),
        "count_mismatch": dict(good, points=good["points"][:2]),
    }
    cfg = {"collections": [{"name": "docs", "dim": 64, "dtype": "bf16"}]}
    for tag, side in bad.items():
        (tmp_path / "docs.points.json").write_text(json.dumps(side))
        eng = pkg.VectorEngine(device=0)
        s = svcmod.VectorService(eng, cfg)
        try:
            with pytest.raises(pkg.VSError) as ei:
                s.restore(str(tmp_path))
            assert ei.value.code in (-8,), (tag, ei.value)
            assert eng.collection_info("docs")["rows"] == 0, tag
            # still a working, empty collection
            st, body, _ = s.handle("POST", "/search", json.dumps(
                {"collection": "docs", "query": [0.1] * 64, "top_k": 3}).encode())
            assert (st, json.loads(body)) == (200, {"results": [], "count": 0}), tag
        finally:
            s.close()
            eng.close()
    # the untouched sidecar still restores
    (tmp_path / "docs.points.json").write_text(json.dumps(good))
    eng = pkg.VectorEngine(device=0)
    s = svcmod.VectorService(eng, cfg)
    try:
        s.restore(str(tmp_path))
        assert eng.collection_info("docs")["rows"] == 103
    finally:
        s.close()
        eng.close()
