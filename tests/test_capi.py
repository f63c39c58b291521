"""The C-ABI boundary without a GPU: every symbol include/eigkl.h declares is
exported by libeigkl_hip.so, the public structs have the layout the Python
mirror assumes, the library carries gfx950 code, GPU entry points fail cleanly
when no device is present, and the drop-in CLIs' argument/file error paths
(cEIG.cpp:143-175, cKL.cpp:431-444) behave like the reference's."""
import ctypes
import os
import re
import subprocess

import pytest

from conftest import PKG_DIR, REPO, circuit_path

HEADER = os.path.join(REPO, "include", "eigkl.h")
LIB = os.path.join(PKG_DIR, "build", "libeigkl_hip.so")


def _declared():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(ek_[a-z0-9_]+)\s*\(", text)))


def test_every_declared_symbol_is_exported(ek):
    names = _declared()
    assert len(names) >= 35
    lib = ctypes.CDLL(LIB)
    missing = [s for s in names if not hasattr(lib, s)]
    assert not missing, missing


def test_struct_layout_matches_python_mirror(ek, tmp_path):
    src = tmp_path / "layout.c"
    src.write_text(
        '#include <stdio.h>\n#include <stddef.h>\n#include "eigkl.h"\n'
        "int main(void) {\n"
        '  printf("%zu %zu %zu %zu\\n", sizeof(ek_swap), sizeof(ek_kl_result), sizeof(ek_lanczos_opts),'
        " sizeof(ek_lanczos_stats));\n"
        '  printf("%zu %zu %zu\\n", offsetof(ek_kl_result, best_iter), offsetof(ek_lanczos_stats, residual),'
        " offsetof(ek_lanczos_opts, reorth));\n"
        "  return 0;\n}\n")
    exe = tmp_path / "layout"
    subprocess.check_call(["gcc", "-std=c99", "-I", os.path.join(REPO, "include"), str(src), "-o", str(exe)])
    a, b = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.splitlines()
    sizes = [int(x) for x in a.split()]
    offs = [int(x) for x in b.split()]
    assert sizes == [ek.SWAP_DTYPE.itemsize, ctypes.sizeof(ek.KLResult), ctypes.sizeof(ek.LanczosOpts),
                     ctypes.sizeof(ek.LanczosStats)]
    assert offs == [ek.KLResult.best_iter.offset, ek.LanczosStats.residual.offset, ek.LanczosOpts.reorth.offset]


def test_library_carries_gfx950_code_only():
    blob = open(LIB, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob
    for other in (b"--gfx942", b"--gfx90a", b"--gfx1100", b"sm_90"):
        assert other not in blob


def test_version(ek):
    assert ek.version()
    # the structs carry no size field; the ABI number the header
    # declares is what the library reports and what the ctypes mirror follows
    import re
    hdr = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "eigkl.h")).read()
    declared = int(re.search(r"#define EIGKL_ABI_VERSION (\d+)", hdr).group(1))
    assert ek._lib.ek_abi_version() == declared == ek.ABI_VERSION


def test_gpu_entry_fails_cleanly_without_device(ek):
    if ek.device_count() > 0:
        pytest.skip("a GPU is present; covered by the gpu suite")
    with pytest.raises(ek.EKError) as e:
        ek.Context(0)
    assert e.value.code == ek.EK_EHIP
    assert "no HIP device" in str(e.value)


def _tool(name):
    return os.path.join(PKG_DIR, "build", "bin", name)


def test_cli_usage_errors(tmp_path):
    r = subprocess.run([_tool("cEIG")], cwd=tmp_path, capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and "Usage" in r.stderr
    r = subprocess.run([_tool("cKL")], cwd=tmp_path, capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and "Usage" in r.stdout  # cKL.cpp:431-434 prints usage on stdout
    r = subprocess.run([_tool("cKL"), "a.hgr", "-EIG", "extra"], cwd=tmp_path, capture_output=True, text=True,
                       timeout=60)
    assert r.returncode == 1
    # both tools create the output directories first (cEIG.cpp:148-149)
    assert (tmp_path / "results").is_dir() and (tmp_path / "pre_saved_EIG").is_dir()


def test_cli_file_errors(tmp_path):
    r = subprocess.run([_tool("cKL"), "missing.hgr"], cwd=tmp_path, capture_output=True, text=True, timeout=60)
    assert r.returncode == 1
    r = subprocess.run([_tool("cEIG"), "missing.hgr"], cwd=tmp_path, capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and "Error" in r.stderr
    # -EIG without pre_saved_EIG/<base>_out.txt: reference exits 1 before any KL work
    r = subprocess.run([_tool("cKL"), circuit_path("fract"), "-EIG"], cwd=tmp_path, capture_output=True, text=True,
                       timeout=60)
    assert r.returncode == 1 and "EIG file not found" in r.stderr
