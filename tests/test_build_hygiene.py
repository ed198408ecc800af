"""Build hygiene: the product build cannot carry experiment defines.

* The Makefile's product rule takes no extra defines, and a change of the compile line (a flags
  stamp rewritten at parse time) makes every object out of date -- so `make all` after an
  experiment-flavoured build rebuilds the product.  Checked on a scratch copy of the Makefile
  with `make -q` and a no-op compiler (no hipcc run).
* Every translation unit records its command-line GF_* defines (gf_buildtag.hpp); the in-tree
  library reports none (`gf_build_is_product`), and experiment hooks refuse to compile without
  GF_EXPERIMENT_BUILD.
"""
import os
import shutil
import subprocess
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "spatialflink_amd", "csrc")


def _make_q(tree, *extra):
    """make -q on the library target: 0 = up to date, 1 = would rebuild."""
    r = subprocess.run(["make", "-q", "-C", tree, "HIPCC=true", "spatialflink_amd/libgeoflink_hip.so", *extra],
                       capture_output=True, text=True)
    assert r.returncode in (0, 1), r.stderr
    return r.returncode


def _touch_all(paths):
    now = time.time()
    for p in paths:
        os.makedirs(os.path.dirname(p), exist_ok=True)
        with open(p, "a"):
            pass
        os.utime(p, (now, now))


def test_makefile_product_rule_has_no_extra_defines():
    mk = open(os.path.join(ROOT, "Makefile")).read()
    assert "GF_DEFS" not in mk
    rule = mk[mk.index("$(OBJDIR)/%.o: $(SRC)/%"):].split("\n\n")[0]
    assert "$(FLAGS_STAMP)" in rule.split("\n")[0], "objects must depend on the flags stamp"
    assert "-D" not in rule


def test_flags_change_rebuilds_and_plain_make_restores_product(tmp_path):
    tree = str(tmp_path)
    shutil.copy(os.path.join(ROOT, "Makefile"), tree)
    # the sources and headers as empty files (make only compares timestamps)
    srcs = [os.path.join(tree, "spatialflink_amd", "csrc", f) for f in os.listdir(SRC)]
    _touch_all(srcs + [os.path.join(tree, "include", "geoflink_hip.h")])
    time.sleep(0.05)
    _make_q(tree)  # parse once: writes the stamp for the default flags
    time.sleep(0.05)
    objs = [os.path.join(tree, "build", "obj", f + ".o") for f in os.listdir(SRC)
            if f.endswith((".cpp", ".hip"))]
    _touch_all(objs + [os.path.join(tree, "spatialflink_amd", "libgeoflink_hip.so")])
    assert _make_q(tree) == 0, "a product build with unchanged flags is up to date"
    # an experiment-flavoured compile line: everything is out of date
    exp = "HIPFLAGS=-O3 --offload-arch=gfx950 -DGF_RANGE_EXP=1"
    assert _make_q(tree, exp) == 1
    time.sleep(0.05)
    _touch_all(objs + [os.path.join(tree, "spatialflink_amd", "libgeoflink_hip.so")])  # "built" that way
    assert _make_q(tree, exp) == 0
    time.sleep(0.05)
    # the next plain `make` sees the product flags again and rebuilds every object
    assert _make_q(tree) == 1
    stamp = open(os.path.join(tree, "build", "obj", ".hipflags")).read()
    assert "-DGF_" not in stamp


def test_experiment_hooks_need_the_experiment_define(tmp_path):
    src = tmp_path / "t.cpp"
    src.write_text('#define GF_TU_NAME t\n#include "gf_buildtag.hpp"\nint main() { return 0; }\n')
    base = ["g++", "-std=c++17", "-fsyntax-only", f"-I{SRC}", str(src)]
    assert subprocess.run(base, capture_output=True).returncode == 0
    r = subprocess.run(base + ["-DGF_RANGE_EXP=1"], capture_output=True, text=True)
    assert r.returncode != 0 and "GF_EXPERIMENT_BUILD" in r.stderr
    assert subprocess.run(base + ["-DGF_RANGE_EXP=1", "-DGF_EXPERIMENT_BUILD"], capture_output=True).returncode == 0


def test_every_unit_records_its_tag():
    for f in os.listdir(SRC):
        if f.endswith((".cpp", ".hip")):
            text = open(os.path.join(SRC, f)).read()
            first = text[text.index("#define GF_TU_NAME"):].split("\n")[:2]
            assert first[0] == f"#define GF_TU_NAME {f.replace('.', '_')}", f
            assert first[1].startswith('#include "gf_buildtag.hpp"'), f
            assert "#include" not in text[:text.index("#define GF_TU_NAME")], f"{f}: tag must come first"


@pytest.mark.skipif(not os.path.exists(os.path.join(ROOT, "spatialflink_amd", "libgeoflink_hip.so")),
                    reason="library not built")
def test_in_tree_library_is_the_product():
    from conftest import assert_product_build

    if os.environ.get("GF_LIB_PATH"):
        pytest.skip("GF_LIB_PATH selects another library")
    info = assert_product_build()
    assert "none (product)" in info
