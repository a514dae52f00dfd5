// PlyLoader.h -- mesh ingestion for the drop-in host API.
//
// Replaces the Assimp import of loadMeshes (src/main.cxx:427-510; Assimp is
// fetched from the network by BuildASSIMP.cmake:22-42 and is not available
// offline).  Reads PLY files (ascii, binary little/big endian; any scalar
// types for x/y/z and for the face index list), fan-triangulates polygons
// (aiProcess_Triangulate, main.cxx:439) and drops faces with fewer than three
// indices (main.cxx:498).  The result is one mesh: vertices (xyz f32) and
// indices (3 per triangle), ready for TriangleMesh::setGeometry(v, idx).
#pragma once

#include <string>
#include <vector>

struct PlyMesh {
    std::vector<float> vertices;       // 3 per vertex
    std::vector<unsigned int> indices; // 3 per triangle
};

// Throws std::runtime_error on I/O or format errors.
PlyMesh loadPly(const std::string& file_name);

// Wavefront OBJ: one mesh per object / group with faces (ObjLoader.cpp).
std::vector<PlyMesh> loadObj(const std::string& file_name);
