"""The C ABI from a plain C host (tests/c_host/orl_host_demo.c): the header compiles as C11, the program links
liborleans_route.so (and the oracle as its checker), and on a GPU it runs the call sequence of a P/Invoke silo —
silo table, ring, registrations, orl_route_batch on page-locked host arrays, orl_route_batch_device on buffers
allocated through the library — bit-exact against the oracle, with no Python on the path."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _build(out_dir):
    gcc = shutil.which("gcc")
    if gcc is None:
        pytest.skip("no gcc")
    lib_dir, ora_dir = os.path.join(ROOT, "orleans_amd"), os.path.join(ROOT, "oracle")
    for f in (os.path.join(lib_dir, "liborleans_route.so"), os.path.join(ora_dir, "liborleans_cpu_ref.so")):
        assert os.path.exists(f), f"{f} not built (make)"
    exe = os.path.join(out_dir, "orl_host_demo")
    cmd = [gcc, "-std=c11", "-O2", "-Wall", "-Wextra", "-Werror", "-I", os.path.join(ROOT, "include"),
           os.path.join(ROOT, "tests", "c_host", "orl_host_demo.c"), "-L", lib_dir, "-lorleans_route", "-L", ora_dir,
           "-lorleans_cpu_ref", f"-Wl,-rpath,{lib_dir}", f"-Wl,-rpath,{ora_dir}", "-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return exe


def test_c_host_compiles_and_links(tmp_path):
    _build(str(tmp_path))


def _keyext_cases(path):
    """The golden KeyExt cases (tests/golden/jenkins.json) as the C host reads them: tcd n0 n1 uniform hex-utf8."""
    import json
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "jenkins.json")))
    with open(path, "w") as f:
        for c in g["keyext"]:
            x = c["ext"].encode("utf-8").hex() or "-"
            f.write(f"{c['tcd']} {c['n0']} {c['n1']} {c['uniform']} {x}\n")
    return len(g["keyext"])


@pytest.mark.gpu
def test_c_host_routes_bit_exact(tmp_path):
    """Steps 1-4 and, with the golden KeyExt cases, step 5: orl_dir_insert_keyext / orl_route_keyext_device from C
    (GrainDirectoryPartition.cs:270-287,326-344, UniqueKey.cs:288-294)."""
    exe = _build(str(tmp_path))
    cases = str(tmp_path / "keyext_cases.txt")
    nk = _keyext_cases(cases)
    r = subprocess.run([exe, cases], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "c host ok" in r.stdout
    assert f"c host KeyExt ok: {nk} golden KeyExt grains registered and {2 * nk} messages routed bit-exact" in r.stdout
