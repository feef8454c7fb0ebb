"""One process per GPU behind the C-ABI: vs_comm_unique_id / vs_comm_init /
vs_gather_merge_keys (include/vsearch.h "one process per GPU").

The one-GPU box holds one rank, so the communicator has one member and RCCL's
all-gather is a copy; the merge after it and the stream ordering are the
product's. Two row shards are searched by one engine each (row_base = the
shard's first global row), their lists concatenated on the device stand in
for the gathered buffer of two ranks and vs_merge_keys of that is checked
against the oracle; vs_gather_merge_keys must equal the merge of its own one
list (a truncation to k). The multi-rank exchange over xGMI is the driver's
8-GPU run (bench.py, VS_COLLECTIVE=engine). Reference anchor: Points.Search,
rag/vector-service/main.go:249-254.
"""
import pytest

pytestmark = pytest.mark.gpu

_COMM = r"""
import sys, json
sys.path.insert(0, ROOT)
import numpy as np, torch
import __graft_entry__ as ge
from oracle import oracle as orc
pkg = ge.load_package()
out = {}
n, dim, nq, kin, k = 120_000, 768, 64, 16, 10
eng = pkg.VectorEngine(device=0)
# errors before the communicator exists
d = torch.zeros((nq, kin), dtype=torch.int64, device="cuda")
o = torch.zeros((nq, k), dtype=torch.int64, device="cuda")
try:
    eng.gather_merge_keys(d.data_ptr(), nq, kin, k, o.data_ptr(), 0)
    out["no_init"] = "accepted"
except pkg.VSError as e:
    out["no_init"] = e.code
uid = pkg.VectorEngine.comm_unique_id()
out["uid_len"] = len(uid)
try:
    eng.comm_init(1, 1, uid)
    out["bad_rank"] = "accepted"
except pkg.VSError as e:
    out["bad_rank"] = e.code
multi = pkg.VectorEngine(shards=[0, 0])
try:
    multi.comm_init(1, 0, uid)
    out["multi"] = "accepted"
except pkg.VSError as e:
    out["multi"] = e.code
multi.close()
eng.comm_init(1, 0, uid)
try:
    eng.comm_init(1, 0, uid)
    out["twice"] = "accepted"
except pkg.VSError as e:
    out["twice"] = e.code
# two row shards, one engine (collection) each, row_base = global first row
half = n // 2
eng.create_collection("s0", dim, 1, 1, half, 0)
eng.create_collection("s1", dim, 1, 1, n - half, half)
eng.generate("s0", half, orc.SEED_CORPUS)
eng.generate("s1", n - half, orc.SEED_CORPUS)
st = torch.cuda.Stream()
with torch.cuda.stream(st):
    dq = torch.empty((nq, dim), dtype=torch.float32, device="cuda")
    eng.generate_vectors(orc.SEED_QUERY, 0, nq, dim, dq.data_ptr(), st.cuda_stream)
    lists = torch.zeros((2, nq, kin), dtype=torch.int64, device="cuda")
    eng.search_keys("s0", dq.data_ptr(), nq, dim, kin, lists[0].data_ptr(), st.cuda_stream)
    eng.search_keys("s1", dq.data_ptr(), nq, dim, kin, lists[1].data_ptr(), st.cuda_stream)
    merged = torch.zeros((nq, k), dtype=torch.int64, device="cuda")
    eng.merge_keys(lists.data_ptr(), 2, nq, kin, k, merged.data_ptr(), st.cuda_stream)
    g = torch.zeros((nq, k), dtype=torch.int64, device="cuda")
    for _ in range(3):  # the gather buffer is reused call to call
        eng.gather_merge_keys(lists[1].data_ptr(), nq, kin, k, g.data_ptr(), st.cuda_stream)
    s, r, c = eng.decode_keys(merged.data_ptr(), nq, k, st.cuda_stream)
st.synchronize()
out["gather_is_truncation"] = bool(torch.equal(g, lists[1, :, :k]))
# (r05) exchanges on two streams, small-k and large-k (> kMaxK, the merge on
# the primary context's scratch) interleaved: every exchange orders itself
# after the previous one on the shared gather buffer, whatever its stream
kbig, kout = 1100, 1050
st2 = torch.cuda.Stream()
with torch.cuda.stream(st):
    big = torch.zeros((nq, kbig), dtype=torch.int64, device="cuda")
    eng.search_keys("s1", dq.data_ptr(), nq, dim, kbig, big.data_ptr(), st.cuda_stream)
st.synchronize()
gb = [torch.zeros((nq, kout), dtype=torch.int64, device="cuda") for _ in range(4)]
gs = [torch.zeros((nq, k), dtype=torch.int64, device="cuda") for _ in range(4)]
for i in range(4):
    sx = st if i % 2 == 0 else st2
    eng.gather_merge_keys(big.data_ptr(), nq, kbig, kout, gb[i].data_ptr(), sx.cuda_stream)
    eng.gather_merge_keys(lists[0].data_ptr(), nq, kin, k, gs[i].data_ptr(), sx.cuda_stream)
torch.cuda.synchronize()
out["two_stream_big"] = all(bool(torch.equal(x, big[:, :kout])) for x in gb)
out["two_stream_small"] = all(bool(torch.equal(x, lists[0, :, :k])) for x in gs)
Qp = orc.preprocess(orc.generate(orc.SEED_QUERY, 0, nq, dim), False, True)
s64, rr, cc = orc.search_generated(orc.SEED_CORPUS, 0, n, Qp, k, True)
resc = orc.rescore_generated(orc.SEED_CORPUS, Qp, r, c, True)
out["bad"] = orc.check_topk(s, r, c, s64, rr, cc, resc, 1e-5)[:5]
eng.close()
print(json.dumps(out))
"""


def test_comm_one_rank():
    from test_gpu_parity import _run_py
    r = _run_py(_COMM)
    assert r["uid_len"] == 128
    assert r["no_init"] == -1 and r["bad_rank"] == -1 and r["multi"] == -1
    assert r["twice"] == -6  # VS_ERR_EXISTS
    assert r["gather_is_truncation"]
    assert r["two_stream_big"] and r["two_stream_small"]
    assert r["bad"] == []
