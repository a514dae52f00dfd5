"""Host code under AddressSanitizer + UBSan.

tools/san_check.sh runs the whole CPU suite over the sanitizer builds
(make SAN=1: simpleraytracing_amd/lib/san/libxrt_host.so + xrt_main,
oracle/san/liboracle.so).  This test runs the part of it that exercises the
host API's own code -- the PLY/OBJ loaders, camera and bbox, Ray::intersect,
the image writers (text, TGA, PGM, JPEG), the CLI -- and the oracle's
golden render and hole fill, so a CPU run of the suite also sees them
sanitised.  The reference's UB sites (main-pthreads-redo.cxx:771's missing
return, Image.inl:209-211's out-of-bounds applyLUT reads) have no analogue
here: both are restated without the bug.
"""
from __future__ import annotations

import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("gcc") is None, reason="no gcc")
def test_host_code_under_asan_ubsan():
    subset = ["tests/test_abi.py::" + t for t in (
        "test_load_ply_matches_oracle", "test_load_ply_errors", "test_ascii_ply_and_quads",
        "test_bbox_and_camera_match_oracle", "test_host_ray_intersect_kat_matches_oracle",
        "test_obj_scene_loading", "test_scene_camera_differs_from_mesh0_camera", "test_jpeg_writer",
        "test_image_writers", "test_cli_help_and_bad_option", "test_cli_without_gpu_reports_error")]
    subset += ["tests/test_oracle.py::test_golden_128_text_byte_exact", "tests/test_oracle.py::test_hole_fill_vs_python_restatement",
               "tests/test_dropin.py"]
    r = subprocess.run([os.path.join(ROOT, "tools", "san_check.sh"), "-x", "-W", "ignore", *subset],
                       cwd=ROOT, capture_output=True, text=True, timeout=900)
    tail = (r.stdout + r.stderr)[-4000:]
    assert r.returncode == 0, tail
    assert "AddressSanitizer" not in tail and "runtime error" not in tail, tail
