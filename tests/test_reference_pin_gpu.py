"""The HIP render path against the REFERENCE kernel's own output on MI355X.

tests/golden/*.npz carry the packed BGR frames the reference kernel produced
(see tests/golden/make_golden.py) in two builds of volumeRender.cl:
  ref_default -- the build the reference host makes (clBuildProgram with no options,
                 RayTracer.cpp:2173);
  ref_strict  -- -cl-fp32-correctly-rounded-divide-sqrt -ffp-contract=off.
The default arithmetic (S_ref) must reproduce ref_default pixel for pixel, S_hw
(RT_FLAG_HW_MATH) must reproduce ref_strict pixel for pixel, and S_strict (the
CPU oracle's arithmetic, RT_FLAG_STRICT_MATH) must agree wherever the oracle does
(the oracle is pinned separately in test_oracle_golden.py).
"""
import numpy as np
import pytest

from conftest import golden_names, load_golden

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", golden_names())
def test_default_math_reproduces_reference_build(renderer, name):
    """rt_render with flags 0 == the reference kernel as RayTracer.cpp builds it."""
    import rtamd
    d = load_golden(name)
    renderer.upload(rtamd.Scene.from_arrays(d))
    renderer.set_params(d["params"])
    w, h = int(d["w"]), int(d["h"])
    out = renderer.render(w, h, depth=int(d["depth"]))
    ndiff = int(np.sum(out != d["ref_default"]))
    print(f"{name}: S_ref vs reference(default build) differing pixels: {ndiff} / {out.size}")
    assert ndiff == 0
    # the wavefront path in the same arithmetic
    wf = renderer.render(w, h, depth=int(d["depth"]), flags=rtamd.RT_FLAG_WAVEFRONT | rtamd.RT_FLAG_WF_SORT)
    assert int(np.sum(wf != d["ref_default"])) == 0


@pytest.mark.parametrize("name", golden_names())
def test_hw_math_reproduces_reference_kernel(renderer, name):
    import rtamd
    d = load_golden(name)
    renderer.upload(rtamd.Scene.from_arrays(d))
    renderer.set_params(d["params"])
    w, h = int(d["w"]), int(d["h"])
    out = renderer.render(w, h, depth=int(d["depth"]), flags=rtamd.RT_FLAG_HW_MATH)
    ndiff = int(np.sum(out != d["ref_strict"]))
    print(f"{name}: S_hw vs reference(strict) differing pixels: {ndiff} / {out.size}")
    assert ndiff == 0


@pytest.mark.parametrize("name", golden_names())
def test_strict_math_close_to_reference_kernel(renderer, name):
    import rtamd
    d = load_golden(name)
    renderer.upload(rtamd.Scene.from_arrays(d))
    renderer.set_params(d["params"])
    out = renderer.render(int(d["w"]), int(d["h"]), depth=int(d["depth"]), flags=rtamd.RT_FLAG_STRICT_MATH)
    assert np.mean(out == d["ref_strict"]) >= 0.999


def test_reference_kernel_rerun_is_stable():
    """Re-run the reference kernel itself (oracle/_ref, when it travelled with the
    snapshot) and check the committed golden is what it produces."""
    import os
    import subprocess
    import sys
    from oracle import ref_ocl
    if not ref_ocl.available():
        pytest.skip("oracle/_ref not built in this snapshot")
    # separate process: the OpenCL runtime must not share this process with torch's HIP runtime
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = ("import sys, numpy as np; sys.path.insert(0, %r); from oracle import ref_ocl; "
            "d = dict(np.load(%r)); out = ref_ocl.render(d, d['params'], int(d['w']), int(d['h']), 'strict'); "
            "print(int(np.sum(out != d['ref_strict'])))" % (root, os.path.join(root, "tests", "golden", "knot16k.npz")))
    res = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert res.returncode == 0, res.stderr
    assert res.stdout.strip().splitlines()[-1] == "0"
