"""The vector-service mirror's JSON layer on CPU: Go encoding/json output rules
and the request decode/validation of searchHandler / upsertHandler
(rag/vector-service/main.go:157-159, :233-237 → 400 "Invalid request body").

Expected strings are what Go's json.Encoder writes (Go >= 1.22) for the same
decoded value: sorted map keys, shortest float64 ('e' form only below 1e-6 or
from 1e21, "e-07" cleaned to "e-7"), <>& and U+2028/9 escaped, '\\n' appended.
"""
import pytest


@pytest.fixture(scope="module")
def svc(pkg):
    from importlib import import_module
    return import_module(pkg.__name__ + ".service")


@pytest.mark.parametrize("doc,want", [
    (b'{"b":1,"a":[1.5,"x<y"],"c":null}', b'{"a":[1.5,"x\\u003cy"],"b":1,"c":null}\n'),
    (b'0.8999999761581421', b'0.8999999761581421\n'),
    (b'1e-7', b'1e-7\n'),
    (b'1.5e-7', b'1.5e-7\n'),
    (b'0.000001', b'0.000001\n'),
    (b'1e21', b'1e+21\n'),
    (b'1e20', b'100000000000000000000\n'),
    (b'123e300', b'1.23e+302\n'),
    (b'-0', b'-0\n'),
    (b'5', b'5\n'),
    (b'5.000', b'5\n'),
    (b'"a&b>c"', b'"a\\u0026b\\u003ec"\n'),
    (b'"\\u2028\\u2029"', b'"\\u2028\\u2029"\n'),
    (b'"\\u0001\\b\\f\\n\\r\\t\\"\\\\/"', b'"\\u0001\\b\\f\\n\\r\\t\\"\\\\/"\n'),
    (b'"caf\\u00e9 \xc3\xa9"', b'"caf\xc3\xa9 \xc3\xa9"\n'),
    (b'"\\ud83d\\ude00"', b'"\xf0\x9f\x98\x80"\n'),
    (b'"\\ud83d"', b'"\xef\xbf\xbd"\n'),
    (b'"bad \xff byte"', b'"bad \xef\xbf\xbd byte"\n'),
    (b'{"k":1,"k":2}', b'{"k":2}\n'),
    (b'{"z":{"y":[true,false,{}],"x":[]}}', b'{"z":{"x":[],"y":[true,false,{}]}}\n'),
    (b'  [1, 2]  trailing', b'[1,2]\n'),
    (b'01', b'0\n'),  # json.Decoder.Decode stops after the first value ("0")
])
def test_go_encoding(svc, doc, want):
    rc, out = svc.reencode(doc)
    assert rc == 0, out
    assert out == want


@pytest.mark.parametrize("doc", [b"", b"{", b"[1,]", b"{'a':1}", b"1.", b".5", b"+1",
                                 b'"\x01"', b"nul", b'{"a" 1}', b"[1 2]", b"-"])
def test_syntax_errors(svc, doc):
    rc, out = svc.reencode(doc)
    assert rc == -1 and out


@pytest.mark.parametrize("body,ok", [
    (b'{"collection":"c","query":[0.1,0.2],"top_k":3}', True),
    (b'{"collection":"c","query":[0.1,0.2],"top_k":3,"filter":{"a":"b"}}', True),
    (b'{"Collection":"c","QUERY":[1],"Top_K":2}', True),          # Go: case-insensitive fields
    (b'{"query":[1,null,2]}', True),                                # null element: zero, no error
    (b'null', True),
    (b'{"query":null,"filter":null,"top_k":null}', True),
    (b'{"collection":"c","query":[1],"unknown":{"x":[1,2]}}', True),
    (b'{"query":[1]} garbage after the first value', True),
    (b'{"top_k":-3}', True),
    (b'', False),
    (b'not json', False),
    (b'[1,2]', False),
    (b'{"query":"abc"}', False),
    (b'{"query":[1,"2"]}', False),
    (b'{"query":[1e39]}', False),                                   # float32 overflow
    (b'{"top_k":5.0}', False),                                      # not an int literal
    (b'{"top_k":1e2}', False),
    (b'{"top_k":"5"}', False),
    (b'{"top_k":99999999999999999999}', False),
    (b'{"filter":[1]}', False),
    (b'{"filter":{"x":1e999}}', False),
    (b'{"collection":5}', False),
])
def test_search_decode(svc, body, ok):
    rc, msg = svc.validate("/search", body)
    assert (rc == 0) == ok, msg


@pytest.mark.parametrize("body,ok", [
    (b'{"collection":"c","points":[{"id":"x","vector":[1,2],"payload":{"text":"t"}}]}', True),
    (b'{"collection":"c","points":[null]}', True),
    (b'{"collection":"c","points":null}', True),
    (b'{"collection":"c"}', True),
    (b'{"collection":"c","points":[1]}', False),
    (b'{"collection":"c","points":{}}', False),
    (b'{"collection":"c","points":[{"vector":[1e400]}]}', False),
    (b'{"collection":["c"]}', False),
    (b'nope', False),
])
def test_upsert_decode(svc, body, ok):
    rc, msg = svc.validate("/upsert", body)
    assert (rc == 0) == ok, msg


def test_service_requires_engine(svc, pkg):
    # without a GPU there is no engine to serve: construction fails loudly
    if pkg.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(pkg.VSError):
        pkg.VectorEngine(device=0)


def _decode(L, body, path):
    import ctypes
    import json
    out = ctypes.c_void_p()
    assert L.vsvc_debug_decode_search(body, len(body), path, ctypes.byref(out)) == 0
    d = json.loads(ctypes.string_at(out.value))
    L.vsvc_free(out)
    return d


def test_search_fast_decoder_matches_generic(svc):
    """The /search fast path (vector_service.cpp decode_search_fast) against
    the generic decoder on typical retrieval-service bodies (it must take
    them, and agree bit for bit) and on bodies it must hand to the generic
    decoder (it must decline them, never answer differently)."""
    import ctypes
    import random
    import numpy as np
    L = svc.load_service_library()
    L.vsvc_debug_decode_search.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int,
                                           ctypes.POINTER(ctypes.c_void_p)]
    rnd = random.Random(11)
    rng = np.random.default_rng(11)

    def num(x):
        f = rnd.randrange(7)
        if f == 0:
            return "%.9g" % x
        if f == 1:
            return repr(float(x))
        if f == 2:
            return "%.17e" % x
        if f == 3:
            return "%dE%+d" % (rnd.randrange(-99999, 99999), rnd.randrange(-30, 30))
        if f == 4:
            return str(rnd.randrange(-3, 3))
        if f == 5:
            return "-0.0e-0"
        return "%.3f" % x

    def ws():
        return rnd.choice(["", " ", "\n  ", "\t", "\r\n"])

    taken = 0
    for t in range(400):
        q = rng.standard_normal(rnd.choice([0, 1, 3, 768])) * 10.0 ** rnd.randrange(-3, 3)
        parts = {"collection": '"%s"' % rnd.choice(["regulatory_docs", "kyc_docs", "", "a b-c_9"]),
                 "query": "[" + ",".join(ws() + num(x) + ws() for x in q) + "]",
                 "top_k": str(rnd.choice([0, 5, 10, -3, 1024, 2 ** 40])),
                 "filter": "null"}
        keys = [k for k in parts if rnd.random() < 0.9]
        rnd.shuffle(keys)
        body = ("{" + ",".join(ws() + '"%s"' % k + ws() + ":" + ws() + parts[k] + ws()
                               for k in keys) + "}" + rnd.choice(["", " ", "\n", "junk"])).encode()
        if not keys:
            body = b"{}"
        fast, gen = _decode(L, body, 1), _decode(L, body, 0)
        if fast != {"error": "declined"}:
            taken += 1
            assert fast == gen, body[:200]
        elif keys:
            pytest.fail(f"fast path declined a typical body: {body[:200]!r}")
    assert taken > 350
    declined = [
        b'{"Query":[1],"top_k":3}', b'{"query":[1],"query":[2]}', b'{"query":[1,null]}',
        b'{"query":null}', b'{"collection":"a\\u0062"}', b'{"collection":"caf\xc3\xa9"}',
        b'{"query":[1e39]}', b'{"query":[1e-50]}', b'{"top_k":1.5}', b'{"top_k":1e2}',
        b'{"top_k":01}', b'{"query":[01]}', b'{"query":[+1]}', b'{"query":[.5]}',
        b'{"query":[1.]}', b'{"filter":{"a":"b"}}', b'{"extra":1}', b'{"query":[1,]}',
        b'{"top_k":99999999999999999999}', b'[1]', b'', b'{', b'{"query":[1]', b'{}',
        b'{"collection":"x","collection":"y"}', b'{"top_k":"5"}', b'{"query":"abc"}']
    for body in declined:
        assert _decode(L, body, 1) == {"error": "declined"}, body
