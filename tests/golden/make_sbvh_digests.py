"""Records SHA-256 digests of the SBVH oracle's output (nodes + tri_indices bytes).

cubes2_obj is the reference's own mesh (x64/Release/data/models/cubes2.obj,
read here as data); its node / ref counts match the survey's probe of the real
SplitBVHBuilder (14,933 / 23,836).  The synthetic meshes are test_sbvh.py's.

    python tests/golden/make_sbvh_digests.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "real-time-opencl-raytracer_amd"), ROOT, os.path.join(ROOT, "tests")]

import rtamd  # noqa: E402
from oracle import oracle  # noqa: E402
from test_sbvh import CUBES2, _meshes, digest  # noqa: E402


def main():
    out = {}
    meshes = dict(_meshes())
    meshes["cubes2_obj"] = lambda: rtamd.Mesh.load_obj(CUBES2)
    for name, make in sorted(meshes.items()):
        a = make().arrays()
        nodes, refs = oracle.sbvh(a["vertices"], a["indices"])
        out[name] = digest(nodes, refs)
        print(name, len(nodes), len(refs), out[name][:16])
    json.dump(out, open(os.path.join(HERE, "sbvh_digests.json"), "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
