"""The C++ drop-in's declarations against the reference's (CPU, no GPU).

INTEGRATION.md claims two things a maintainer of the reference relies on:

* its ``src/main-cuda.cxx`` binding compiles against the reference's own
  headers (``include/Vec3.h``, ``TriangleMesh.h``, ``Image.h`` ...) and this
  repo's C ABI (``include/xrt.h``);
* code written against ``src/main.cxx``'s declarations (``RayTracerInfo``
  ``:111-121`` and the prototypes ``:126-161``) compiles against the host API
  (``simpleraytracing_amd/csrc/host``), ``renderLoop`` returning ``void``.

Both tests read the reference's source text from /root/reference (skipped
where it is absent -- the GPU box has no copy) and compile with
``g++ -std=c++11`` only; nothing of the reference is copied into the repo or
run.
"""
from __future__ import annotations

import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
MAIN = os.path.join(REF, "src", "main.cxx")
HOST = os.path.join(ROOT, "simpleraytracing_amd", "csrc", "host")

needs_reference = pytest.mark.skipif(not os.path.isfile(MAIN), reason="the reference sources are not here")


def main_cxx_lines(first, last):
    """Lines first..last (1-based, inclusive) of the reference's src/main.cxx."""
    with open(MAIN, encoding="utf-8", errors="replace") as f:
        lines = f.read().splitlines()
    return "\n".join(lines[first - 1:last]) + "\n"


def declarations():
    """RayTracerInfo and the function declarations of main.cxx (:111-161),
    checked to be what this test expects to be there."""
    text = main_cxx_lines(111, 161)
    assert text.lstrip().startswith("struct RayTracerInfo"), text[:80]
    assert "void renderLoop(Image& anOutputImage," in text
    return text


def integration_snippet():
    with open(os.path.join(ROOT, "INTEGRATION.md"), encoding="utf-8") as f:
        md = f.read()
    blocks = re.findall(r"```cpp\n(.*?)```", md, flags=re.S)
    snippet = [b for b in blocks if b.startswith("// src/main-cuda.cxx")]
    assert len(snippet) == 1, "INTEGRATION.md holds one main-cuda.cxx binding"
    return snippet[0]


def compile_tu(tmp_path, source, includes):
    tu = tmp_path / "tu.cxx"
    tu.write_text(source)
    cmd = ["g++", "-std=c++11", "-c", "-o", str(tmp_path / "tu.o"), "-Wall", "-Wno-unused-variable",
           "-Wno-unused-but-set-variable"] + [f"-I{d}" for d in includes] + [str(tu)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, f"{' '.join(cmd)}\n{r.stderr[-4000:]}"


@needs_reference
def test_integration_binding_compiles_against_reference_headers(tmp_path):
    """INTEGRATION.md's main-cuda.cxx, in the translation unit main.cxx makes
    (its standard headers, the reference's own Vec3/Ray/TriangleMesh/Material/
    Image headers, RayTracerInfo and the prototypes), against include/xrt.h."""
    head = "".join(f"#include <{h}>\n" for h in ("iostream", "exception", "algorithm", "cmath", "limits",
                                                 "stdexcept", "sstream", "string", "chrono", "vector",
                                                 "cstdint"))
    head += "".join(f'#include "{h}"\n' for h in ("Vec3.h", "Ray.h", "TriangleMesh.h", "Material.h", "Image.h",
                                                  "Light.h"))
    src = head + "using namespace std;\n" + declarations() + integration_snippet()
    compile_tu(tmp_path, src, [os.path.join(REF, "include"), os.path.join(ROOT, "include")])


@needs_reference
def test_reference_declarations_compile_against_host_api(tmp_path):
    """main.cxx's prototypes (:126-161), verbatim, next to the host API's
    declarations of the same functions: any difference in a return or
    parameter type is a compile error.  RayTracerInfo has the reference's
    members, in its order."""
    protos = main_cxx_lines(126, 161)
    assert protos.lstrip().startswith("void showUsage"), protos[:60]
    use = """
#include <cstddef>
void use_members(RayTracerInfo& info)
{
    Vec3* members[] = {&info.detector_position, &info.origin, &info.up, &info.right,
                       &info.upper_bbox_corner, &info.lower_bbox_corner, &info.range};
    Light& light = info.light;
    static_assert(offsetof(RayTracerInfo, right) < offsetof(RayTracerInfo, light) &&
                  offsetof(RayTracerInfo, light) < offsetof(RayTracerInfo, upper_bbox_corner),
                  "RayTracerInfo members in main.cxx:111-121's order");
    (void)members;
    (void)light;
}
void (*const render_loop)(Image&, const vector<TriangleMesh>&, RayTracerInfo&) = renderLoop;
void (*const get_bbox)(const vector<TriangleMesh>&, Vec3&, Vec3&) = getBBox;
void (*const load_meshes)(const std::string&, vector<TriangleMesh>&) = loadMeshes;
RayTracerInfo (*const init)(vector<TriangleMesh>&, const Vec3&, const Vec3&, const unsigned int,
                            const unsigned int, Image&, float) = initialiseRayTracing;
"""
    src = '#include "RayTracer.h"\n#include <string>\nusing namespace std;\n' + protos + use
    compile_tu(tmp_path, src, [HOST, os.path.join(ROOT, "include")])
