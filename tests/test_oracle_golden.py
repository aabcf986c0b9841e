"""Pin the CPU oracle to the REFERENCE kernel's own output.

tests/golden/<name>.npz holds, for each fixture, the raytracer_bvh inputs and
the packed BGR frame the reference kernel (x64/Release/volumeRender.cl,
compiled for gfx950 by oracle/Makefile.ref, run on MI355X through the ROCm
OpenCL runtime by tests/golden/make_golden.py) produced for them:
  ref_strict  -- reference built with correctly rounded '/' + sqrt, no contraction
  ref_default -- reference built with the options its host uses (clBuildProgram "")

The oracle's S_strict arithmetic differs from the strict build only in
normalize()'s rsqrt and GGX's pow (hardware approximations in the device
library), so a handful of pixels may differ; the bar below is the
measured agreement, and the GPU test test_reference_pin_gpu.py shows the HIP
kernel in S_hw mode reproduces ref_strict exactly.
"""
import numpy as np
import pytest

from conftest import golden_names, load_golden

MIN_EXACT_STRICT = 0.999      # fraction of pixels identical to ref_strict, per fixture
MIN_EXACT_DEFAULT = 0.99      # vs the default (contracting, approximate-division) build
EXACT_STRICT = {"cornell12_orbit", "overflow_comb", "rand2k", "rand3k_bigleaf", "single_tri_rootleaf",
                "sphere_obj", "bad_node"}


def _oracle_out(d):
    from oracle import oracle
    return oracle.render(d, d["params"], int(d["w"]), int(d["h"]), depth=int(d["depth"]), nthreads=8)


@pytest.mark.parametrize("name", golden_names())
def test_oracle_matches_reference_kernel(name):
    d = load_golden(name)
    assert "ref_strict" in d, "fixture lacks the reference kernel output (run make_golden.py reference + merge)"
    out = _oracle_out(d)["out"]
    strict = np.mean(out == d["ref_strict"])
    default = np.mean(out == d["ref_default"])
    print(f"{name}: exact vs ref_strict {strict:.6f}, vs ref_default {default:.6f}")
    assert strict >= MIN_EXACT_STRICT
    assert default >= MIN_EXACT_DEFAULT
    if name in EXACT_STRICT:
        assert strict == 1.0


def test_overall_agreement():
    tot = same = 0
    for name in golden_names():
        d = load_golden(name)
        out = _oracle_out(d)["out"]
        tot += out.size
        same += int(np.sum(out == d["ref_strict"]))
    assert same / tot >= 0.9995, same / tot


def test_overflow_fixture_is_all_miss():
    """The 70-deep comb BVH overflows the 65-entry stack -> every traced pixel black
    in the reference kernel (volumeRender.cl:914) and in the oracle."""
    d = load_golden("overflow_comb")
    r = _oracle_out(d)
    assert np.all(d["ref_strict"] == 0)
    assert np.all(r["out"] == 0)
    assert r["stats"]["stack_overflow"] > 0


def test_bad_node_fixture_has_misses():
    d = load_golden("bad_node")
    r = _oracle_out(d)
    assert np.array_equal(r["out"], d["ref_strict"])
