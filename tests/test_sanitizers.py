"""Host code and the CPU oracle under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY.md 5:
sanitizers on the CPU side; GPU sanitizers are not available on this pool).

tests/sanitize_main.cpp drives the scene generators, the OBJ / Collada loaders, the SBVH and
binned builders, the BVH cache and the camera (csrc/host/*.cpp, the same sources librtamd.so
is built from, compiled here with g++) and the oracle (oracle/*.c), with every sanitizer
report fatal (-fno-sanitize-recover=all).  It also checks the product SBVH against the SBVH
oracle byte for byte and the oracle's frames across thread counts."""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT

PKG = os.path.join(ROOT, "real-time-opencl-raytracer_amd")
HOST = ["scene.cpp", "bvh_builder.cpp", "sbvh_builder.cpp", "collada.cpp", "rt_host_abi.cpp"]
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-g", "-O1"]

OBJ = """# two triangles with normals, one without
v -10 0 -10
v 10 0 -10
v 10 0 10
v -10 0 10
v 0 15 0
vn 0 1 0
f 1//1 2//1 3//1
f 1//1 3//1 4//1
f 1 2 5
"""


@pytest.fixture(scope="module")
def sanitized_driver(tmp_path_factory):
    if not (shutil.which("gcc") and shutil.which("g++")):
        pytest.skip("gcc/g++ not available")
    out = tmp_path_factory.mktemp("san")
    objs = []
    for c in ("rt_oracle.c", "sbvh_oracle.c"):
        o = str(out / (c + ".o"))
        subprocess.run(["gcc", "-std=c11", "-ffp-contract=off", "-fno-fast-math", *SAN, "-c",
                        os.path.join(ROOT, "oracle", c), "-o", o], check=True, timeout=300)
        objs.append(o)
    srcs = [os.path.join(PKG, "csrc", "host", s) for s in HOST] + [os.path.join(ROOT, "tests", "sanitize_main.cpp")]
    procs = []
    for s in srcs:
        o = str(out / (os.path.basename(s) + ".o"))
        procs.append(subprocess.Popen(["g++", "-std=c++17", "-ffp-contract=off", *SAN, "-I", os.path.join(ROOT, "include"),
                                       "-I", os.path.join(PKG, "csrc", "host"), "-c", s, "-o", o]))
        objs.append(o)
    for p in procs:
        assert p.wait(timeout=600) == 0
    exe = str(out / "sanitize_main")
    subprocess.run(["g++", *SAN, "-o", exe, *objs, "-lpthread", "-lm"], check=True, timeout=300)
    return exe, out


def test_host_code_and_oracle_are_clean_under_asan_ubsan(sanitized_driver):
    exe, out = sanitized_driver
    obj = out / "mesh.obj"
    obj.write_text(OBJ)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    p = subprocess.run([exe, str(out), str(obj)], capture_output=True, text=True, timeout=900, env=env)
    assert p.returncode == 0, (p.stdout[-2000:], p.stderr[-4000:])
    assert "ALL OK" in p.stdout
    assert "runtime error" not in p.stderr and "AddressSanitizer" not in p.stderr, p.stderr[-4000:]
    for name in ("cornell", "knot", "heightfield", "grid", "random", "obj"):
        assert f"{name}:" in p.stdout
