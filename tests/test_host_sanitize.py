"""Host-side sanitizer configuration: the library's host
code built with AddressSanitizer + UndefinedBehaviorSanitizer
(tools/sanitize/Makefile, -fsanitize after -Xarch_host; device code unchanged)
and driven by tools/sanitize/host_check.cpp without a GPU: the tile planner,
shape choice and workspace carving over widths 5..256, rectangles, batches
1..256, every op and layout, plus every argument-validation path."""

import os
import subprocess

from conftest import ROOT


def test_host_code_under_asan_ubsan():
    env = dict(os.environ)
    env.pop("IRLMX_PLAN_CUS", None)
    r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tools", "sanitize"), "-j8", "run"],
                       capture_output=True, text=True, env=env, timeout=900)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "host_check ok" in out, out[-4000:]
    assert "ERROR: AddressSanitizer" not in out and "runtime error" not in out, out[-4000:]
