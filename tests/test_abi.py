"""The C-ABI boundary on CPU: the library loads, exports every function
include/vsearch.h declares, refuses to run without a GPU (no CPU fallback),
and the documented key layout sorts like (score desc, row asc)."""
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "vsearch.h")


def declared_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    names = set(re.findall(r"^\s*(?:const\s+)?[A-Za-z_][\w\s\*]*?\b(vs_\w+)\s*\(", txt, re.M))
    inline = set(re.findall(r"static inline [\w\s\*]+?\b(vs_\w+)\s*\(", txt))
    return sorted(names - inline)


def test_header_compiles_as_c_and_cpp(tmp_path):
    src = tmp_path / "t.c"
    src.write_text('#include "vsearch.h"\nint main(void){return vs_key_row(vs_key_encode(1.0f, 7u)) == 7u ? 0 : 1;}\n')
    for cc, ext in (("gcc", "c"), ("g++", "cpp")):
        f = tmp_path / f"t.{ext}"
        f.write_text(src.read_text())
        exe = tmp_path / f"t_{ext}"
        subprocess.run([cc, "-Wall", "-Werror", "-I", os.path.dirname(HEADER), str(f), "-o", str(exe)],
                       check=True)
        assert subprocess.run([str(exe)]).returncode == 0


def test_library_exports_every_declared_symbol(pkg):
    L = pkg.load_library()
    decl = declared_functions()
    assert len(decl) >= 15
    for name in decl:
        assert hasattr(L, name), f"{name} not exported"
    from importlib import import_module
    eng_mod = import_module(pkg.__name__ + ".engine")
    assert sorted(eng_mod.EXPORTS) == decl


def test_service_library_exports_every_declared_symbol(pkg):
    import ctypes
    from importlib import import_module
    svc = import_module(pkg.__name__ + ".service")
    L = svc.load_service_library()
    txt = re.sub(r"/\*.*?\*/", "", open(os.path.join(ROOT, "include", "vsearch_service.h")).read(),
                 flags=re.S)
    names = sorted(set(re.findall(r"^\s*[A-Za-z_][\w\s\*]*?\b(vsvc_\w+)\s*\(", txt, re.M)))
    assert {"vsvc_open", "vsvc_handle", "vsvc_snapshot", "vsvc_restore", "vsvc_loadgen",
            "vsvc_stats", "vsvc_bulk_generate"} <= set(names)
    for name in names:
        assert hasattr(L, name), f"{name} not exported"
    assert isinstance(L, ctypes.CDLL)


def test_library_links_only_the_hip_runtime(pkg):
    out = subprocess.run(["ldd", pkg.load_library()._name], capture_output=True, text=True).stdout
    assert "libamdhip64" in out
    assert "oracle" not in out and "torch" not in out


def test_no_gpu_fails_loudly(pkg):
    if pkg.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(pkg.VSError) as ei:
        pkg.VectorEngine(device=0)
    assert ei.value.code == -5  # VS_ERR_DEVICE
    assert "no CPU fallback" in ei.value.msg


def test_key_layout_orders_like_score_desc_row_asc(tmp_path, pkg):
    rng = np.random.default_rng(1)
    scores = np.concatenate([rng.standard_normal(200).astype(np.float32),
                             np.array([0.0, -0.0, 1.0, 1.0, -1.0, 3.4e38, -3.4e38], np.float32)])
    rows = rng.integers(0, 2 ** 32 - 2, scores.shape[0]).astype(np.uint32)
    rows[-5:] = [5, 9, 3, 4, 4]
    prog = tmp_path / "keys.c"
    vals = ",".join(f"{s!r}f" if np.isfinite(s) else "0.0f" for s in scores.tolist())
    rws = ",".join(f"{r}u" for r in rows.tolist())
    prog.write_text(f'''#include <stdio.h>
#include "vsearch.h"
static const float S[] = {{{vals}}};
static const unsigned R[] = {{{rws}}};
int main(void) {{ for (unsigned i = 0; i < sizeof(S)/sizeof(S[0]); ++i)
  printf("%llu\\n", (unsigned long long)vs_key_encode(S[i], R[i])); return 0; }}
''')
    exe = tmp_path / "keys"
    subprocess.run(["gcc", "-I", os.path.dirname(HEADER), str(prog), "-o", str(exe)], check=True)
    keys = np.array([int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True).stdout.split()],
                    dtype=np.uint64)
    ds, dr, cnt = pkg.keys_decode(keys[None, :])
    assert np.array_equal(ds[0], scores) or np.array_equal(ds[0][scores != 0], scores[scores != 0])
    assert np.array_equal(dr[0], rows.astype(np.uint64))
    by_key = np.argsort(-keys.astype(np.float64), kind="stable")  # float64 loses bits: use python sort
    by_key = sorted(range(len(keys)), key=lambda i: int(keys[i]), reverse=True)
    by_rule = sorted(range(len(keys)), key=lambda i: (-float(scores[i]), int(rows[i])))
    # +0.0 / -0.0 compare equal by score but differ in key; compare the rest
    assert [i for i in by_key if scores[i] != 0] == [i for i in by_rule if scores[i] != 0]


def test_build_id_is_the_tree_hash(pkg):
    """The loaded library was linked from exactly the sources of this tree."""
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "_vs_build_t", os.path.join(os.path.dirname(pkg.__file__), "build.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    bid = pkg.build_id()
    assert re.fullmatch(r"[0-9a-f]{16}", bid)
    assert bid == b.tree_hash()


def test_copy_last_error_is_the_same_call_message(pkg):
    """vs_copy_last_error (the cgo wrappers' single-call read) returns the
    thread's last failure text, truncated and NUL-terminated."""
    import ctypes
    L = pkg.load_library()
    rc = L.vs_open(None, None)  # out == NULL -> invalid argument
    assert rc == -1
    full = L.vs_last_error()
    assert full
    buf = ctypes.create_string_buffer(256)
    n = L.vs_copy_last_error(buf, len(buf))
    assert n == len(full) and buf.value == full
    small = ctypes.create_string_buffer(5)
    assert L.vs_copy_last_error(small, 5) == len(full)
    assert small.value == full[:4]
    assert L.vs_copy_last_error(None, 0) == len(full)


_RT_PROBE = r"""
import json, os, sys
sys.path.insert(0, {root!r})
import __graft_entry__ as ge
pkg = ge.load_package()
L = pkg.load_library()
import torch  # noqa: F401  (after the library: a second runtime unless load_library imported it first)
from importlib import import_module
eng = import_module(pkg.__name__ + ".engine")
rc = L.vs_runtime_check()
print(json.dumps({{"rc": rc, "msg": L.vs_last_error().decode() if rc else "",
                  "runtimes": eng.hip_runtimes()}}))
"""


@pytest.mark.parametrize("torch_first", ["1", "0"])
def test_one_hip_runtime_per_process(torch_first):
    """Regression for the round-3 driver failure: torch's
    wheel bundles its own libamdhip64.so, so loading libvsearch before torch
    mapped two HIP runtimes whose streams are unordered with each other.
    load_library now imports torch first (one runtime); with that disabled
    the library's own check refuses device-pointer calls (VS_ERR_DEVICE)."""
    import json
    env = dict(os.environ, VS_TORCH_FIRST=torch_first)
    out = subprocess.run([os.sys.executable, "-c", _RT_PROBE.format(root=ROOT)], env=env,
                         capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    r = json.loads(out.stdout.strip().splitlines()[-1])
    if torch_first == "1":
        assert len(r["runtimes"]) == 1, r
        assert r["rc"] == 0
    else:
        assert len(r["runtimes"]) == 2, r
        assert r["rc"] == -5 and "two HIP runtimes" in r["msg"], r
