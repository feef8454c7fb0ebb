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
