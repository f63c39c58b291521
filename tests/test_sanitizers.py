"""ASan + UBSan build of the product's host code (SURVEY §5 "race detection /
sanitizers"): hgr.cpp, graph_build.cpp, io.cpp, host_linalg.cpp, common.cpp,
solve.cpp and cli.cpp compiled by g++ with -fsanitize=address,undefined
(-fno-sanitize-recover: any UB report fails), linked with a helper standing in
for the GPU-side entry points as a machine without a gfx950 device sees them
(tests/helpers/gpu_absent.cpp), and driven over the shipped circuits, the
generator, edge-case and malformed inputs, and the CLI error paths
(tests/helpers/host_sanitize.cpp).  CPU only."""
import os
import subprocess

import pytest

from conftest import GOLD, PKG_DIR, REPO

SRC = os.path.join(PKG_DIR, "csrc")
HOST = ["common.cpp", "hgr.cpp", "graph_build.cpp", "io.cpp", "host_linalg.cpp", "solve.cpp", "cli.cpp"]


@pytest.mark.timeout(600)
def test_host_code_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "host_sanitize")
    srcs = [os.path.join(SRC, f) for f in HOST] + [os.path.join(REPO, "tests", "helpers", f) for f in
                                                   ("gpu_absent.cpp", "host_sanitize.cpp")]
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-pthread",
                           "-fsanitize=address,undefined", "-fno-sanitize-recover=all", *srcs, "-o", exe])
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1",
               EK_THREADS="4")
    r = subprocess.run([exe, GOLD, str(tmp_path)], cwd=tmp_path, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "host sanitize ok" in r.stdout
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr
