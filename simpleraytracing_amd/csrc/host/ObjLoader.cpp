// ObjLoader.cpp -- Wavefront OBJ scenes for the drop-in loadMeshes (see
// PlyLoader.h).  The reference imports every mesh of a file through Assimp
// (src/main.cxx:455-508); an OBJ file is how a multi-object scene reaches it.
//
// One mesh per object: a new mesh starts at each `o` or `g` line that follows
// faces (empty groups make no mesh), in file order, so mesh 0 -- the only one
// whose hits count, main.cxx:687 -- is the file's first object with faces.
// Vertices (`v x y z [w]`) are global to the file; face corners are `i`,
// `i/t`, `i//n` or `i/t/n`, 1-based or negative (relative to the vertices read
// so far); polygons are fan-triangulated (aiProcess_Triangulate, :439) and
// faces with fewer than three corners dropped (:498).  Other statements
// (vt, vn, usemtl, mtllib, s, l, p, comments) are ignored.  Assimp's own OBJ
// splitting (one mesh per object and material) is not restated: parity of the
// mesh boundaries is unpinned (DESIGN.md "Multi-mesh scenes").
#include "PlyLoader.h"

#include <cstdlib>
#include <fstream>
#include <sstream>
#include <stdexcept>

namespace {

[[noreturn]] void fail(const std::string& file, size_t line, const std::string& what)
{
    throw std::runtime_error("OBJ " + file + ":" + std::to_string(line) + ": " + what);
}

}  // namespace

std::vector<PlyMesh> loadObj(const std::string& file_name)
{
    std::ifstream in(file_name);
    if (!in) throw std::runtime_error("Cannot open " + file_name);
    std::vector<float> vertices;                 // 3 per vertex, the whole file
    std::vector<std::vector<unsigned int>> faces(1);
    std::string text;
    size_t line_no = 0;
    while (std::getline(in, text)) {
        ++line_no;
        std::istringstream ls(text);
        std::string tag;
        if (!(ls >> tag) || tag[0] == '#') continue;
        if (tag == "v") {
            float x, y, z;
            if (!(ls >> x >> y >> z)) fail(file_name, line_no, "vertex needs x y z");
            vertices.push_back(x);
            vertices.push_back(y);
            vertices.push_back(z);
        } else if (tag == "o" || tag == "g") {
            if (!faces.back().empty()) faces.emplace_back();
        } else if (tag == "f") {
            std::vector<unsigned int> corners;
            std::string c;
            while (ls >> c) {
                char* end = nullptr;
                const long v = std::strtol(c.c_str(), &end, 10);
                if (end == c.c_str() || (*end != '\0' && *end != '/')) fail(file_name, line_no, "bad face corner " + c);
                const long n = (long)(vertices.size() / 3);
                const long idx = v > 0 ? v - 1 : n + v;
                if (v == 0 || idx < 0 || idx >= n) fail(file_name, line_no, "vertex index out of range: " + c);
                corners.push_back((unsigned int)idx);
            }
            for (size_t k = 1; k + 1 < corners.size(); ++k) {   // fan, as aiProcess_Triangulate
                faces.back().push_back(corners[0]);
                faces.back().push_back(corners[k]);
                faces.back().push_back(corners[k + 1]);
            }
        }
    }
    std::vector<PlyMesh> meshes;
    for (auto& f : faces) {
        if (f.empty()) continue;
        PlyMesh m;
        m.vertices = vertices;
        m.indices = std::move(f);
        meshes.push_back(std::move(m));
    }
    return meshes;
}
