"""The cgo package's C preamble (go/vsearch/vsearch.go) compiles as C and its
error-capturing wrappers work: no Go toolchain exists in this image, so the
preamble is cut out of the Go file, compiled with gcc against
include/vsearch.h, linked with libvsearch.so and driven from C. Each vsg_*
wrapper must hand back the failing call's message from the same C call (the
cgo error-capture rule: vs_last_error() is thread-local and a goroutine may
change OS threads between two cgo calls)."""
import os
import re
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GO_FILE = os.path.join(ROOT, "go", "vsearch", "vsearch.go")


def preamble() -> str:
    src = open(GO_FILE).read()
    m = re.search(r"/\*\n(#cgo.*?)\*/\nimport \"C\"", src, re.S)
    assert m, "cgo preamble not found"
    return "\n".join(l for l in m.group(1).splitlines() if not l.startswith("#cgo"))


def test_every_engine_call_goes_through_a_wrapper():
    src = open(GO_FILE).read()
    body = src[src.index('import "C"'):]
    direct = set(re.findall(r"C\.(vs_\w+)\(", body)) - {"vs_close"}
    assert not direct, f"direct cgo calls without error capture: {sorted(direct)}"
    wrappers = set(re.findall(r"C\.(vsg_\w+)\(", body))
    defined = set(re.findall(r"static int (vsg_\w+)\(", preamble()))
    assert wrappers <= defined
    assert "C.vs_last_error" not in body


def test_preamble_compiles_and_captures_the_message(tmp_path, pkg):
    lib = pkg.load_library()._name
    c = tmp_path / "pre.c"
    c.write_text(preamble() + r'''
#include <stdio.h>
#include <string.h>
int main(void) {
  vsg_err e; memset(&e, 0, sizeof e);
  int rc = vsg_open(NULL, NULL, &e);           /* out == NULL: invalid argument */
  if (rc != VS_ERR_INVALID_ARG || e.msg[0] == 0) return 1;
  printf("%s\n", e.msg);
  vsg_err ok; memset(&ok, 0, sizeof ok);
  if (vsg_fin(0, &ok) != 0 || ok.msg[0] != 0) return 2;  /* success leaves it empty */
  return 0;
}
''')
    exe = tmp_path / "pre"
    subprocess.run(["gcc", "-std=c11", "-Wall", "-Werror", "-Wno-unused-function",
                    "-I", os.path.join(ROOT, "include"), str(c), "-o", str(exe), lib,
                    "-Wl,-rpath," + os.path.dirname(lib)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True)
    assert r.returncode == 0, r
    assert "out is NULL" in r.stdout  # vs_open's own message, read in the same call
