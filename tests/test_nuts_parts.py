"""The NUTS kernel instantiations are spread over nuts_part0.hip ...
nuts_part5.hip (nuts_launch.h); every layout of GM_LAYOUT_LIST (gm_layouts.h)
must be compiled in exactly one part, or nuts_run would reject that layout
(or two parts would define the same kernels)."""
import os
import re

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "general-mcmc_amd", "csrc")


def _pairs(text):
    return [(int(a), int(b)) for a, b in re.findall(r"X\((\d+),\s*(\d+)\)", text)]


def test_every_layout_in_exactly_one_nuts_part():
    with open(os.path.join(CSRC, "gm_layouts.h")) as f:
        src = f.read()
    block = src[src.index("#define GM_LAYOUT_LIST(X)"):src.index("namespace gm")]
    layouts = _pairs(block)
    assert len(layouts) == len(set(layouts)) and layouts
    seen = []
    for k in range(6):
        with open(os.path.join(CSRC, f"nuts_part{k}.hip")) as f:
            part = f.read()
        line = next(l for l in part.splitlines() if l.startswith("#define GM_NUTS_PART_LAYOUTS"))
        assert f"#define GM_NUTS_PART {k}" in part
        seen += _pairs(line)
    assert sorted(seen) == sorted(layouts)


def test_parts_are_built_and_dispatched():
    with open(os.path.join(CSRC, "..", "Makefile")) as f:
        mk = f.read()
    with open(os.path.join(CSRC, "nuts_launch.h")) as f:
        launch = f.read()
    for k in range(6):
        assert f"csrc/nuts_part{k}.hip" in mk
        assert f"nuts_launch_part{k}," in launch or f"nuts_launch_part{k}}}" in launch
