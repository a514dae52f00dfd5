/*
 * xrt_oracle.c -- TEST INFRASTRUCTURE ONLY.  Not product code.
 *
 * A plain-C, CPU restatement of the reference's X-ray attenuation render path
 * (Brandagot/SimpleRayTracing).  It is the checker the GPU path is compared
 * against: only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * may load it.  The product path (libxrt.so) never links or calls it.
 *
 * Every function cites the reference file:line it restates.  Floating-point
 * evaluation order, the float/double mix and the libm calls follow the
 * reference exactly (build with -O2 -ffp-contract=off, no -ffast-math):
 *   - f32 '+', '-', '*', '/' and sqrtf are correctly rounded on x86-64;
 *   - (float)(1.0/(double)det) is kept as written (src/Ray.cxx:99);
 *   - expf is glibc's expf, the function std::exp(float) binds to.
 *
 * Pinned by (see tests/test_oracle.py):
 *   - tests/golden/dragon-128x128-serial.txt: the reference's own golden output
 *     (out/dragon-128x128-serial.txt), reproduced byte for byte;
 *   - Ray::intersect known-answer vectors produced by oracle/_ref, i.e. the
 *     reference's unmodified src/Ray.cxx compiled in this container.
 */
#define _GNU_SOURCE
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define ORC_OK 0
#define ORC_ERR_IO 1
#define ORC_ERR_FORMAT 2
#define ORC_ERR_ARG 3

/* ------------------------------------------------------------------------- */
/* Vec3 helpers: include/Vec3.inl                                            */
/* ------------------------------------------------------------------------- */

/* Vec3::crossProduct, include/Vec3.inl:321-329 */
static inline void cross3(const float a[3], const float b[3], float out[3])
{
    float x = a[1] * b[2] - a[2] * b[1];
    float y = a[2] * b[0] - a[0] * b[2];
    float z = a[0] * b[1] - a[1] * b[0];
    out[0] = x;
    out[1] = y;
    out[2] = z;
}

/* Vec3::dotProduct, include/Vec3.inl:313-317 -- ((x*x') + (y*y')) + (z*z') */
static inline float dot3(const float a[3], const float b[3])
{
    return a[0] * b[0] + a[1] * b[1] + a[2] * b[2];
}

/* Vec3::getLength, include/Vec3.inl:461-465 (std::sqrt(float) -> sqrtf) */
static inline float length3(const float a[3])
{
    return sqrtf(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]);
}

/* Vec3::normalise, include/Vec3.inl:469-476 */
static inline void normalise3(float a[3])
{
    float len = length3(a);
    a[0] /= len;
    a[1] /= len;
    a[2] /= len;
}

/* ------------------------------------------------------------------------- */
/* Ray::intersect, src/Ray.cxx:72-124 (Moller-Trumbore, non-culling)         */
/* ------------------------------------------------------------------------- */
int orc_intersect(const float origin[3], const float direction[3],
                  const float p1[3], const float p2[3], const float p3[3],
                  float* t_out)
{
    float edge1[3] = {p2[0] - p1[0], p2[1] - p1[1], p2[2] - p1[2]}; /* :86 */
    float edge2[3] = {p3[0] - p1[0], p3[1] - p1[1], p3[2] - p1[2]}; /* :87 */
    float pvec[3];
    cross3(direction, edge2, pvec);                                   /* :90 */
    float det = dot3(edge1, pvec);                                    /* :93 */
    if (fpclassify(det) == FP_ZERO) return 0;                         /* :94 */
    float inv_det = (float)(1.0 / (double)det);                       /* :99 */
    float tvec[3] = {origin[0] - p1[0], origin[1] - p1[1], origin[2] - p1[2]}; /* :102 */
    float u = dot3(tvec, pvec) * inv_det;                             /* :105 */
    if ((double)u < 0.0 || (double)u > 1.0) return 0;                 /* :106 */
    float qvec[3];
    cross3(tvec, edge1, qvec);                                        /* :112 */
    float v = dot3(direction, qvec) * inv_det;                        /* :115 */
    if ((double)v < 0.0 || (double)(u + v) > 1.0) return 0;           /* :116 */
    *t_out = dot3(edge2, qvec) * inv_det;                             /* :122 */
    return 1;
}

/*
 * Batched KAT entry: rays[6*i] = origin, direction; tris[9*i] = p1,p2,p3.
 * The direction goes through the Ray ctor first (include/Ray.inl:74-85:
 * divided by its length unless that length is zero), as in the reference.
 */
void orc_intersect_batch(const float* rays, const float* tris, uint64_t n,
                         uint8_t* hit, float* t)
{
    for (uint64_t i = 0; i < n; ++i) {
        float tt = 0.0f;
        const float* dir = rays + 6 * i + 3;
        float d[3] = {0.0f, 0.0f, 0.0f};
        float len = length3(dir);
        if (fpclassify(len) != FP_ZERO) {
            d[0] = dir[0] / len;
            d[1] = dir[1] / len;
            d[2] = dir[2] / len;
        }
        int h = orc_intersect(rays + 6 * i, d, tris + 9 * i,
                              tris + 9 * i + 3, tris + 9 * i + 6, &tt);
        hit[i] = (uint8_t)h;
        t[i] = h ? tt : 0.0f;
    }
}

/* ------------------------------------------------------------------------- */
/* Mesh ingestion: a minimal PLY reader standing in for Assimp's import      */
/* (src/main.cxx:427-510) followed by TriangleMesh::setGeometry(v, idx)      */
/* (src/TriangleMesh.cxx:104-131).  Output is a triangle soup, 9 f32 each.   */
/* ------------------------------------------------------------------------- */
enum ply_type { PT_NONE, PT_I8, PT_U8, PT_I16, PT_U16, PT_I32, PT_U32, PT_F32, PT_F64 };

static enum ply_type ply_parse_type(const char* s)
{
    if (!strcmp(s, "char") || !strcmp(s, "int8")) return PT_I8;
    if (!strcmp(s, "uchar") || !strcmp(s, "uint8")) return PT_U8;
    if (!strcmp(s, "short") || !strcmp(s, "int16")) return PT_I16;
    if (!strcmp(s, "ushort") || !strcmp(s, "uint16")) return PT_U16;
    if (!strcmp(s, "int") || !strcmp(s, "int32")) return PT_I32;
    if (!strcmp(s, "uint") || !strcmp(s, "uint32")) return PT_U32;
    if (!strcmp(s, "float") || !strcmp(s, "float32")) return PT_F32;
    if (!strcmp(s, "double") || !strcmp(s, "float64")) return PT_F64;
    return PT_NONE;
}

static int ply_size(enum ply_type t)
{
    switch (t) {
    case PT_I8: case PT_U8: return 1;
    case PT_I16: case PT_U16: return 2;
    case PT_I32: case PT_U32: case PT_F32: return 4;
    case PT_F64: return 8;
    default: return 0;
    }
}

static double ply_read_bin(const unsigned char* p, enum ply_type t)
{
    switch (t) {
    case PT_I8: return (double)*(const int8_t*)p;
    case PT_U8: return (double)*(const uint8_t*)p;
    case PT_I16: { int16_t v; memcpy(&v, p, 2); return v; }
    case PT_U16: { uint16_t v; memcpy(&v, p, 2); return v; }
    case PT_I32: { int32_t v; memcpy(&v, p, 4); return v; }
    case PT_U32: { uint32_t v; memcpy(&v, p, 4); return v; }
    case PT_F32: { float v; memcpy(&v, p, 4); return v; }
    case PT_F64: { double v; memcpy(&v, p, 8); return v; }
    default: return 0.0;
    }
}

#define PLY_MAX_PROPS 32
struct ply_prop { char name[64]; enum ply_type type; enum ply_type count_type; int is_list; };
struct ply_elem { char name[64]; uint64_t count; int nprops; struct ply_prop props[PLY_MAX_PROPS]; };

/*
 * Loads a PLY file into a triangle soup.  Polygons with more than three
 * vertices are fan-triangulated (Assimp aiProcess_Triangulate, main.cxx:439);
 * faces with fewer than three are dropped (main.cxx:498).
 * On success *tris_out is malloc'd (caller frees with orc_free).
 */
int orc_load_ply(const char* path, float** tris_out, uint64_t* ntris_out)
{
    *tris_out = NULL;
    *ntris_out = 0;
    FILE* f = fopen(path, "rb");
    if (!f) return ORC_ERR_IO;
    fseek(f, 0, SEEK_END);
    long fsize = ftell(f);
    fseek(f, 0, SEEK_SET);
    unsigned char* buf = (unsigned char*)malloc((size_t)fsize + 1);
    if (!buf || fread(buf, 1, (size_t)fsize, f) != (size_t)fsize) {
        fclose(f);
        free(buf);
        return ORC_ERR_IO;
    }
    fclose(f);
    buf[fsize] = 0;

    struct ply_elem elems[8];
    int nelems = 0, binary = -1;
    size_t pos = 0;
    int rc = ORC_ERR_FORMAT;
    float* verts = NULL;
    float* tris = NULL;
    uint64_t ntris = 0, cap = 0;

    if (fsize < 4 || memcmp(buf, "ply", 3) != 0) goto done;
    for (;;) {
        size_t eol = pos;
        while (eol < (size_t)fsize && buf[eol] != '\n') ++eol;
        if (eol >= (size_t)fsize) goto done;
        char line[256];
        size_t len = eol - pos;
        if (len > sizeof(line) - 1) len = sizeof(line) - 1;
        memcpy(line, buf + pos, len);
        line[len] = 0;
        if (len && line[len - 1] == '\r') line[len - 1] = 0;
        pos = eol + 1;
        char a[64] = {0}, b[64] = {0}, c[64] = {0}, d[64] = {0}, e[64] = {0};
        int n = sscanf(line, "%63s %63s %63s %63s %63s", a, b, c, d, e);
        if (n <= 0) continue;
        if (!strcmp(a, "format")) {
            if (!strcmp(b, "binary_little_endian")) binary = 1;
            else if (!strcmp(b, "ascii")) binary = 0;
            else goto done; /* big endian not supported */
        } else if (!strcmp(a, "element")) {
            if (nelems >= 8 || n < 3) goto done;
            memset(&elems[nelems], 0, sizeof(elems[0]));
            snprintf(elems[nelems].name, sizeof elems[nelems].name, "%s", b);
            elems[nelems].count = strtoull(c, NULL, 10);
            ++nelems;
        } else if (!strcmp(a, "property")) {
            if (!nelems) goto done;
            struct ply_elem* el = &elems[nelems - 1];
            if (el->nprops >= PLY_MAX_PROPS) goto done;
            struct ply_prop* pr = &el->props[el->nprops++];
            if (!strcmp(b, "list")) {
                pr->is_list = 1;
                pr->count_type = ply_parse_type(c);
                pr->type = ply_parse_type(d);
                snprintf(pr->name, sizeof pr->name, "%s", e);
            } else {
                pr->type = ply_parse_type(b);
                snprintf(pr->name, sizeof pr->name, "%s", c);
            }
            if (pr->type == PT_NONE || (pr->is_list && pr->count_type == PT_NONE)) goto done;
        } else if (!strcmp(a, "end_header")) {
            break;
        }
    }
    if (binary < 0) goto done;

    uint64_t nverts = 0;
    for (int ei = 0; ei < nelems; ++ei) {
        struct ply_elem* el = &elems[ei];
        int is_vertex = !strcmp(el->name, "vertex");
        int is_face = !strcmp(el->name, "face");
        int ix = -1, iy = -1, iz = -1;
        if (is_vertex) {
            for (int p = 0; p < el->nprops; ++p) {
                if (!strcmp(el->props[p].name, "x")) ix = p;
                if (!strcmp(el->props[p].name, "y")) iy = p;
                if (!strcmp(el->props[p].name, "z")) iz = p;
            }
            if (ix < 0 || iy < 0 || iz < 0) goto done;
            nverts = el->count;
            verts = (float*)malloc(sizeof(float) * 3 * (nverts ? nverts : 1));
            if (!verts) goto done;
        }
        for (uint64_t r = 0; r < el->count; ++r) {
            for (int p = 0; p < el->nprops; ++p) {
                struct ply_prop* pr = &el->props[p];
                if (!pr->is_list) {
                    double val;
                    if (binary) {
                        int sz = ply_size(pr->type);
                        if (pos + sz > (size_t)fsize) goto done;
                        val = ply_read_bin(buf + pos, pr->type);
                        pos += sz;
                    } else {
                        char* endp;
                        val = strtod((const char*)buf + pos, &endp);
                        if (endp == (const char*)buf + pos) goto done;
                        pos = (size_t)(endp - (char*)buf);
                    }
                    if (is_vertex) {
                        if (p == ix) verts[3 * r + 0] = (float)val;
                        if (p == iy) verts[3 * r + 1] = (float)val;
                        if (p == iz) verts[3 * r + 2] = (float)val;
                    }
                } else {
                    uint64_t cnt;
                    if (binary) {
                        int sz = ply_size(pr->count_type);
                        if (pos + sz > (size_t)fsize) goto done;
                        cnt = (uint64_t)ply_read_bin(buf + pos, pr->count_type);
                        pos += sz;
                    } else {
                        char* endp;
                        cnt = strtoull((const char*)buf + pos, &endp, 10);
                        pos = (size_t)(endp - (char*)buf);
                    }
                    uint64_t idx[64];
                    if (cnt > 64) goto done;
                    for (uint64_t k = 0; k < cnt; ++k) {
                        if (binary) {
                            int sz = ply_size(pr->type);
                            if (pos + sz > (size_t)fsize) goto done;
                            idx[k] = (uint64_t)ply_read_bin(buf + pos, pr->type);
                            pos += sz;
                        } else {
                            char* endp;
                            idx[k] = strtoull((const char*)buf + pos, &endp, 10);
                            pos = (size_t)(endp - (char*)buf);
                        }
                    }
                    if (is_face && cnt >= 3 &&
                        (!strcmp(pr->name, "vertex_indices") || !strcmp(pr->name, "vertex_index"))) {
                        for (uint64_t k = 1; k + 1 < cnt; ++k) {
                            uint64_t tri[3] = {idx[0], idx[k], idx[k + 1]};
                            if (ntris == cap) {
                                cap = cap ? cap * 2 : 4096;
                                float* nt = (float*)realloc(tris, sizeof(float) * 9 * cap);
                                if (!nt) goto done;
                                tris = nt;
                            }
                            for (int q = 0; q < 3; ++q) {
                                if (tri[q] >= nverts) goto done;
                                memcpy(tris + 9 * ntris + 3 * q, verts + 3 * tri[q], 3 * sizeof(float));
                            }
                            ++ntris;
                        }
                    }
                }
            }
        }
    }
    rc = ORC_OK;
done:
    free(buf);
    free(verts);
    if (rc == ORC_OK) {
        *tris_out = tris;
        *ntris_out = ntris;
    } else {
        free(tris);
    }
    return rc;
}

void orc_free(void* p) { free(p); }

/* ------------------------------------------------------------------------- */
/* Bounding box: TriangleMesh::computeBoundingBox (src/TriangleMesh.cxx:192- */
/* 228) with std::min/std::max semantics; getBBox (src/main.cxx:538-563).    */
/* ------------------------------------------------------------------------- */
static inline float stdmin(float a, float b) { return (b < a) ? b : a; }
static inline float stdmax(float a, float b) { return (a < b) ? b : a; }

void orc_bbox(const float* tris, uint64_t ntris, float lower[3], float upper[3])
{
    for (int k = 0; k < 3; ++k) {
        lower[k] = INFINITY;
        upper[k] = -INFINITY;
    }
    for (uint64_t i = 0; i < ntris; ++i)
        for (int v = 0; v < 3; ++v)
            for (int k = 0; k < 3; ++k) {
                float x = tris[9 * i + 3 * v + k];
                lower[k] = stdmin(lower[k], x);
                upper[k] = stdmax(upper[k], x);
            }
}

/* ------------------------------------------------------------------------- */
/* Camera: initialiseRayTracing (src/main.cxx:566-622) and the renderLoop    */
/* prologue (src/main.cxx:634-641).                                          */
/* cam[0..2] origin, [3..5] detector, [6..8] up, [9..11] right, [12] ps      */
/* ------------------------------------------------------------------------- */
void orc_camera(const float lower[3], const float upper[3], uint32_t width,
                uint32_t height, float cam[13])
{
    float range[3] = {upper[0] - lower[0], upper[1] - lower[1], upper[2] - lower[2]}; /* :575 */
    float centre[3];
    for (int k = 0; k < 3; ++k)                                        /* :576, Vec3::operator/(double) */
        centre[k] = lower[k] + (float)((double)range[k] / 2.0);
    float diagonal = length3(range);                                   /* :586 */
    float up[3] = {0.0f, 0.0f, -1.0f};                                 /* :588 */
    float origin[3] = {centre[0] - diagonal * 1, centre[1] - 0.0f, centre[2] - 0.0f}; /* :590 */
    float dxoff = (float)((double)diagonal * 0.6);                     /* :591 */
    float detector[3] = {centre[0] + dxoff, centre[1] + 0.0f, centre[2] + 0.0f};
    float direction[3] = {detector[0] - origin[0], detector[1] - origin[1], detector[2] - origin[2]}; /* :593 */
    normalise3(direction);                                             /* :594 */
    normalise3(direction);                                             /* :603 */
    float right[3];
    cross3(direction, up, right);                                      /* :604 */

    /* renderLoop prologue, :637-641 (getBBox again gives the same corners) */
    float res1 = range[2] / (float)width;
    float res2 = range[1] / (float)height;
    float ps = 2 * stdmax(res1, res2);

    memcpy(cam + 0, origin, sizeof origin);
    memcpy(cam + 3, detector, sizeof detector);
    memcpy(cam + 6, up, sizeof up);
    memcpy(cam + 9, right, sizeof right);
    cam[12] = ps;
}

/* ------------------------------------------------------------------------- */
/* renderLoop, src/main.cxx:626-743, over a range of image rows.             */
/* ------------------------------------------------------------------------- */
static int cmp_float(const void* a, const void* b)
{
    float x = *(const float*)a, y = *(const float*)b;
    return (x < y) ? -1 : (x > y) ? 1 : 0;
}

/*
 * 8-bit image: Image::applyLUT's per-pixel formula (include/Image.inl:195-211)
 * with vmin = 0, vmax = 80 (I0), evaluated as written: (v - vmin) in float,
 * then 255.0 * . / (vmax - vmin) in double, round() half away from zero.
 */
static inline uint8_t lut_u8(float v)
{
    const float vmin = 0.0f, vmax = 80.0f;
    if (v < vmin) return 0;
    if (v > vmax) return 255;
    if (v != v) return 0; /* NaN: undefined in the reference; pinned to 0 */
    return (uint8_t)round(255.0 * (v - vmin) / (vmax - vmin));
}

struct render_job {
    const float* tris;       /* the scene's meshes, soups one after another */
    uint64_t ntris;          /* triangles of mesh 0 (the first ntris of tris) */
    const uint64_t* mesh_ntris;  /* triangles per mesh */
    uint32_t nmeshes;
    int signed_model;        /* 1: main-pthreads-lbuffer.cxx's signed L-buffer */
    const float* cam;
    uint32_t width, height;
    const uint32_t* rows;  /* image rows to render, output row i = rows[i] */
    uint32_t nrows;
    float* image;          /* nrows*width, may be NULL */
    float* lbuffer;        /* may be NULL */
    uint8_t* image_u8;     /* may be NULL */
    int32_t* nhits;        /* may be NULL */
    uint32_t col_begin, col_end;  /* columns rendered in every listed row */
    uint64_t next_unit;    /* work unit = 64 consecutive pixels of one row */
    uint64_t units_per_row;
    pthread_mutex_t lock;
    uint64_t odd_rays;
};

static void render_pixel(const struct render_job* job, uint32_t row, uint32_t col,
                         float** hits, size_t* hits_cap, float* img, float* lb,
                         uint8_t* u8, int32_t* nh, uint64_t* odd)
{
    const float* cam = job->cam;
    const float* origin = cam + 0;
    const float* detector = cam + 3;
    const float* up = cam + 6;
    const float* right = cam + 9;
    float ps = cam[12];

    /* :655-656 -- double arithmetic, then narrowed to float */
    float v_offset = (float)((double)ps * (0.5 + (double)row - (double)job->height / 2.0));
    float u_offset = (float)((double)ps * (0.5 + (double)col - (double)job->width / 2.0));

    /* :659 -- detector + up*v + right*u - origin, left to right, f32 */
    float direction[3];
    for (int k = 0; k < 3; ++k)
        direction[k] = ((detector[k] + up[k] * v_offset) + right[k] * u_offset) - origin[k];
    normalise3(direction);                                             /* :660 */

    /* Ray ctor, include/Ray.inl:74-85 -- normalises again */
    float d[3] = {0.0f, 0.0f, 0.0f};
    float len = length3(direction);
    if (fpclassify(len) != FP_ZERO) {
        d[0] = direction[0] / len;
        d[1] = direction[1] / len;
        d[2] = direction[2] / len;
    }

    /* :670-696 -- every mesh (intersectBBox is `return true`, TriangleMesh.inl:
     * 232-236) and every triangle; only hits on mesh 0 with t > 1e-7 (double
     * compare) are kept (:687).  Ray::intersect has no side effects, so the
     * other meshes' tests -- whose results :687 discards -- are skipped. */
    size_t count = 0;
    for (uint32_t m = 0; m < job->nmeshes; ++m) {
        if (m != 0) continue;
        for (uint64_t i = 0; i < job->mesh_ntris[0]; ++i) {
            const float* tr = job->tris + 9 * i;
            float t;
            if (orc_intersect(origin, d, tr, tr + 3, tr + 6, &t) && (double)t > 0.0000001) {
                if (count == *hits_cap) {
                    *hits_cap *= 2;
                    *hits = (float*)realloc(*hits, sizeof(float) * *hits_cap);
                }
                (*hits)[count++] = t;
            }
        }
    }

    /* :700-718 -- L-buffer: sorted pairwise path length, odd count -> 0 */
    float distance = 0;
    float lval = INFINITY; /* z_buffer initial value, :646 */
    if (count > 0) {
        if (count % 2 == 0) {
            qsort(*hits, count, sizeof(float), cmp_float);
            for (size_t i = 0; i < count; i += 2)
                distance += (*hits)[i + 1] - (*hits)[i];
        } else {
            ++*odd; /* "Only one intersect on this ray", :710 */
        }
        lval = distance;
    }

    /* :725, :739 -- Beer-Lambert, std::exp(float) -> expf */
    distance = (float)((double)distance * 0.1);
    float photon = 80.000f * expf(-(0.3971f * distance));

    if (img) *img = photon;
    if (lb) *lb = lval;
    if (u8) *u8 = lut_u8(photon);
    if (nh) *nh = (int32_t)count;
}

/*
 * The signed multi-material L-buffer, src/main-pthreads-lbuffer.cxx:750-811
 * (renderLoopCallBack of the L-buffer fork): per mesh, the sum of
 * sign(direction . normal) * t over mesh-0 hits in triangle order; a non-zero
 * sum of the signs flags the pixel -1 (:805-806), otherwise the L-buffer value
 * (initially 80, :314) is attenuated with the mesh's coefficient (:798-808).
 * Camera and ray as main.cxx (the fork's :739-762 restate :639-661).
 */
static void render_pixel_signed(const struct render_job* job, uint32_t row, uint32_t col, float* lb,
                                int32_t* nh, uint64_t* flagged)
{
    const float* cam = job->cam;
    const float* origin = cam + 0;
    const float* detector = cam + 3;
    const float* up = cam + 6;
    const float* right = cam + 9;
    float ps = cam[12];
    float v_offset = (float)((double)ps * (0.5 + (double)row - (double)job->height / 2.0));  /* :756 */
    float u_offset = (float)((double)ps * (0.5 + (double)col - (double)job->width / 2.0));   /* :757 */
    float direction[3];
    for (int k = 0; k < 3; ++k)                                        /* :760 */
        direction[k] = ((detector[k] + up[k] * v_offset) + right[k] * u_offset) - origin[k];
    normalise3(direction);                                             /* :761 */
    float d[3] = {0.0f, 0.0f, 0.0f};                                   /* :762, Ray ctor */
    float len = length3(direction);
    if (fpclassify(len) != FP_ZERO) {
        d[0] = direction[0] / len;
        d[1] = direction[1] / len;
        d[2] = direction[2] / len;
    }
    float L = 80.000f;                                                 /* :314 */
    int32_t count = 0;
    uint64_t first = 0;
    for (uint32_t m = 0; m < job->nmeshes; ++m) {                      /* :768 */
        const uint64_t n = job->mesh_ntris[m];
        if (L == -1) break;                                            /* :772 */
        float distance = 0.0f;                                         /* :778 */
        int sign_sum = 0;
        for (uint64_t i = 0; m == 0 && i < n; ++i) {                   /* :780; :788 keeps mesh 0 only */
            const float* tr = job->tris + 9 * (first + i);
            float t;
            if (orc_intersect(origin, d, tr, tr + 3, tr + 6, &t) && (double)t > 0.0000001) {
                /* Triangle::computeNormal, include/Triangle.inl:170-178 */
                float e1[3] = {tr[3] - tr[0], tr[4] - tr[1], tr[5] - tr[2]};
                float e2[3] = {tr[6] - tr[0], tr[7] - tr[1], tr[8] - tr[2]};
                float nrm[3];
                cross3(e1, e2, nrm);
                normalise3(nrm);
                float dp = dot3(direction, nrm);                       /* :791 */
                int sign = (0.0f < dp) - (dp < 0.0f);                  /* signum, :729-731 */
                distance += (float)sign * t;                           /* :792 */
                sign_sum += sign;                                      /* :793 */
                ++count;
            }
        }
        float mu = m == 0 ? 0.1037f : 0.3971f;                         /* :798-803 */
        if (sign_sum != 0)
            L = -1;                                                    /* :806 */
        else                                                           /* :808, std::exp(double) */
            L = (float)((double)L * exp(-((double)mu * ((double)distance * 0.1))));
        first += n;
    }
    if (L == -1) ++*flagged;
    if (lb) *lb = L;
    if (nh) *nh = count;
}

static void* render_worker(void* arg)
{
    struct render_job* job = (struct render_job*)arg;
    size_t cap = 64;
    float* hits = (float*)malloc(sizeof(float) * cap);
    uint64_t odd = 0;
    const uint64_t total = job->units_per_row * job->nrows;
    for (;;) {
        pthread_mutex_lock(&job->lock);
        uint64_t unit = job->next_unit++;
        pthread_mutex_unlock(&job->lock);
        if (unit >= total) break;
        uint32_t i = (uint32_t)(unit / job->units_per_row);
        uint32_t span = job->col_end - job->col_begin;
        uint32_t c0 = job->col_begin + (uint32_t)(unit % job->units_per_row) * 64u;
        uint32_t c1 = c0 + 64u < job->col_end ? c0 + 64u : job->col_end;
        size_t base = (size_t)i * span - job->col_begin;
        for (uint32_t col = c0; col < c1; ++col) {
            size_t o = base + col;
            if (job->signed_model) {
                render_pixel_signed(job, job->rows[i], col, job->lbuffer ? job->lbuffer + o : NULL,
                                    job->nhits ? job->nhits + o : NULL, &odd);
                continue;
            }
            render_pixel(job, job->rows[i], col, &hits, &cap,
                         job->image ? job->image + o : NULL,
                         job->lbuffer ? job->lbuffer + o : NULL,
                         job->image_u8 ? job->image_u8 + o : NULL,
                         job->nhits ? job->nhits + o : NULL, &odd);
        }
    }
    pthread_mutex_lock(&job->lock);
    job->odd_rays += odd;
    pthread_mutex_unlock(&job->lock);
    free(hits);
    return NULL;
}

static int64_t render_scene(const float* tris, const uint64_t* mesh_ntris, uint32_t nmeshes, int signed_model,
                            const float cam[13], uint32_t width, uint32_t height, const uint32_t* rows,
                            uint32_t nrows, uint32_t col_begin, uint32_t col_end, float* image,
                            float* lbuffer, uint8_t* image_u8, int32_t* nhits, int nthreads);

static int64_t render_list(const float* tris, uint64_t ntris, const float cam[13], uint32_t width,
                           uint32_t height, const uint32_t* rows, uint32_t nrows,
                           uint32_t col_begin, uint32_t col_end, float* image,
                           float* lbuffer, uint8_t* image_u8, int32_t* nhits, int nthreads)
{
    return render_scene(tris, &ntris, 1, 0, cam, width, height, rows, nrows, col_begin, col_end, image,
                        lbuffer, image_u8, nhits, nthreads);
}

static int64_t render_scene(const float* tris, const uint64_t* mesh_ntris, uint32_t nmeshes, int signed_model,
                            const float cam[13], uint32_t width, uint32_t height, const uint32_t* rows,
                            uint32_t nrows, uint32_t col_begin, uint32_t col_end, float* image,
                            float* lbuffer, uint8_t* image_u8, int32_t* nhits, int nthreads)
{
    const uint64_t no_mesh = 0;
    if (nmeshes == 0) mesh_ntris = &no_mesh;   /* no meshes: nothing is hit */
    for (uint32_t i = 0; i < nrows; ++i)
        if (rows[i] >= height) return -1;
    if (col_begin > col_end || col_end > width) return -1;
    struct render_job job;
    memset(&job, 0, sizeof job);
    job.tris = tris;
    job.ntris = mesh_ntris[0];
    job.mesh_ntris = mesh_ntris;
    job.nmeshes = nmeshes ? nmeshes : 1;
    job.signed_model = signed_model;
    job.cam = cam;
    job.width = width;
    job.height = height;
    job.rows = rows;
    job.nrows = nrows;
    job.image = image;
    job.lbuffer = lbuffer;
    job.image_u8 = image_u8;
    job.nhits = nhits;
    job.col_begin = col_begin;
    job.col_end = col_end;
    job.units_per_row = (col_end - col_begin + 63u) / 64u;
    pthread_mutex_init(&job.lock, NULL);
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    for (int i = 1; i < nthreads; ++i) pthread_create(&th[i], NULL, render_worker, &job);
    render_worker(&job);
    for (int i = 1; i < nthreads; ++i) pthread_join(th[i], NULL);
    pthread_mutex_destroy(&job.lock);
    return (int64_t)job.odd_rays;
}

/*
 * Renders rows [row_begin, row_end) of a width x height image.  Output
 * buffers are strip-relative (index (row-row_begin)*width+col), any may be
 * NULL.  Returns the number of odd-hit-count rays (each of which the
 * reference reports with "Only one intersect on this ray"), or -1.
 */
int64_t orc_render_rows(const float* tris, uint64_t ntris, const float cam[13],
                        uint32_t width, uint32_t height, uint32_t row_begin,
                        uint32_t row_end, float* image, float* lbuffer,
                        uint8_t* image_u8, int32_t* nhits, int nthreads)
{
    if (row_end > height || row_begin > row_end) return -1;
    uint32_t n = row_end - row_begin;
    uint32_t* rows = (uint32_t*)malloc(sizeof(uint32_t) * (n ? n : 1));
    for (uint32_t i = 0; i < n; ++i) rows[i] = row_begin + i;
    int64_t odd = render_list(tris, ntris, cam, width, height, rows, n, 0, width, image, lbuffer,
                              image_u8, nhits, nthreads);
    free(rows);
    return odd;
}

/* Renders an explicit list of rows (strip-boundary samples of large images). */
int64_t orc_render_row_list(const float* tris, uint64_t ntris, const float cam[13],
                            uint32_t width, uint32_t height, const uint32_t* rows,
                            uint32_t nrows, float* image, float* lbuffer,
                            uint8_t* image_u8, int32_t* nhits, int nthreads)
{
    return render_list(tris, ntris, cam, width, height, rows, nrows, 0, width, image, lbuffer,
                       image_u8, nhits, nthreads);
}

/* Columns [col_begin, col_end) of a list of rows (sampled checks of huge frames). */
int64_t orc_render_row_list_span(const float* tris, uint64_t ntris, const float cam[13],
                                 uint32_t width, uint32_t height, const uint32_t* rows,
                                 uint32_t nrows, uint32_t col_begin, uint32_t col_end,
                                 float* image, float* lbuffer, uint8_t* image_u8,
                                 int32_t* nhits, int nthreads)
{
    return render_list(tris, ntris, cam, width, height, rows, nrows, col_begin, col_end, image,
                       lbuffer, image_u8, nhits, nthreads);
}

/* Columns [col_begin, col_end) of one row (bounded CPU timing samples). */
int64_t orc_render_span(const float* tris, uint64_t ntris, const float cam[13], uint32_t width,
                        uint32_t height, uint32_t row, uint32_t col_begin, uint32_t col_end,
                        float* image, float* lbuffer, uint8_t* image_u8, int32_t* nhits,
                        int nthreads)
{
    return render_list(tris, ntris, cam, width, height, &row, 1, col_begin, col_end, image,
                       lbuffer, image_u8, nhits, nthreads);
}

/*
 * A scene of several meshes (tris = their soups one after another,
 * mesh_ntris[m] = triangles of mesh m): renderLoop's mesh loop with the
 * mesh-0 filter (main.cxx:670-696), rows [row_begin, row_end).
 */
int64_t orc_render_scene_rows(const float* tris, const uint64_t* mesh_ntris, uint32_t nmeshes,
                              const float cam[13], uint32_t width, uint32_t height, uint32_t row_begin,
                              uint32_t row_end, float* image, float* lbuffer, uint8_t* image_u8,
                              int32_t* nhits, int nthreads)
{
    if (row_end > height || row_begin > row_end) return -1;
    uint32_t n = row_end - row_begin;
    uint32_t* rows = (uint32_t*)malloc(sizeof(uint32_t) * (n ? n : 1));
    for (uint32_t i = 0; i < n; ++i) rows[i] = row_begin + i;
    int64_t odd = render_scene(tris, mesh_ntris, nmeshes, 0, cam, width, height, rows, n, 0, width, image,
                               lbuffer, image_u8, nhits, nthreads);
    free(rows);
    return odd;
}

/*
 * The signed L-buffer of src/main-pthreads-lbuffer.cxx:733-813 over rows
 * [row_begin, row_end): lbuffer = the fork's L_buffer values (80-based photon
 * counts, or -1 for a flagged pixel), nhits = mesh-0 hits per ray.  Returns
 * the number of flagged pixels, or -1.
 */
int64_t orc_render_signed_rows(const float* tris, const uint64_t* mesh_ntris, uint32_t nmeshes,
                               const float cam[13], uint32_t width, uint32_t height, uint32_t row_begin,
                               uint32_t row_end, float* lbuffer, int32_t* nhits, int nthreads)
{
    if (row_end > height || row_begin > row_end) return -1;
    uint32_t n = row_end - row_begin;
    uint32_t* rows = (uint32_t*)malloc(sizeof(uint32_t) * (n ? n : 1));
    for (uint32_t i = 0; i < n; ++i) rows[i] = row_begin + i;
    int64_t flagged = render_scene(tris, mesh_ntris, nmeshes, 1, cam, width, height, rows, n, 0, width, NULL,
                                   lbuffer, NULL, nhits, nthreads);
    free(rows);
    return flagged;
}

/*
 * The fork's "error correction" pass, src/main-pthreads-lbuffer.cxx:327-404:
 * each pixel flagged -1 becomes the mean of the first unflagged value within
 * 4 steps in each of four directions (+1 and -1 along the row-major index --
 * which runs on into the next / previous row -- and +-1 row), skipping zero
 * values; a pixel with no such value becomes 0.0f / 0 (NaN).  Index
 * arithmetic is the fork's unsigned int arithmetic; an index past the buffer
 * ends the walk.  The fork also reads the element one past the end (its test
 * is `> size`, not `>= size`) -- undefined behaviour, taken here as the end
 * of the walk.  Reads L only (the fill does not cascade), writes image.
 */
void orc_hole_fill(const float* L, uint32_t width, uint32_t height, float* image)
{
    const uint64_t size = (uint64_t)width * height;
    const int max_depth = 4;                                           /* :339 */
    for (uint64_t pixel = 0; pixel < size; ++pixel) {
        uint32_t row = (uint32_t)(pixel / width);
        uint32_t col = (uint32_t)(pixel % width);
        float photon = L[(uint32_t)(row * width + col)];               /* :334 */
        if (photon == -1) {                                            /* :338 */
            float values[4];
            size_t count = 0;
            for (int dir = 0; dir < 4; ++dir) {
                float value = 0;
                for (int i = 1; i <= max_depth; ++i) {
                    uint32_t idx;
                    switch (dir) {
                    case 0: idx = row * width + (col + (uint32_t)i); break;    /* :343-352 */
                    case 1: idx = (row - (uint32_t)i) * width + col; break;    /* :356-365 */
                    case 2: idx = row * width + (col - (uint32_t)i); break;    /* :369-378 */
                    default: idx = (row + (uint32_t)i) * width + col; break;   /* :382-391 */
                    }
                    if ((uint64_t)idx >= size) break;                   /* `> size` + the UB read */
                    if (L[idx] != -1) {
                        value = L[idx];
                        break;
                    }
                }
                if (value != 0) values[count++] = value;
            }
            float sum = 0;                                             /* :394-397 */
            for (size_t k = 0; k < count; ++k) sum += values[k];
            photon = sum / (float)count;                               /* :399 */
        }
        image[pixel] = photon;                                         /* :403 */
    }
}

/* getBBox (main.cxx:538-563) over the meshes' computeBoundingBox boxes. */
void orc_scene_bbox(const float* tris, const uint64_t* mesh_ntris, uint32_t nmeshes, float lower[3],
                    float upper[3])
{
    for (int k = 0; k < 3; ++k) {
        lower[k] = INFINITY;
        upper[k] = -INFINITY;
    }
    uint64_t first = 0;
    for (uint32_t m = 0; m < nmeshes; ++m) {
        float lo[3], hi[3];
        orc_bbox(tris + 9 * first, mesh_ntris[m], lo, hi);
        for (int k = 0; k < 3; ++k) {
            lower[k] = stdmin(lower[k], lo[k]);
            upper[k] = stdmax(upper[k], hi[k]);
        }
        first += mesh_ntris[m];
    }
}

/* Triangle::computeNormal (include/Triangle.inl:170-178) of each triangle. */
void orc_triangle_normals(const float* tris, uint64_t n, float* normals)
{
    for (uint64_t i = 0; i < n; ++i) {
        const float* tr = tris + 9 * i;
        float e1[3] = {tr[3] - tr[0], tr[4] - tr[1], tr[5] - tr[2]};
        float e2[3] = {tr[6] - tr[0], tr[7] - tr[1], tr[8] - tr[2]};
        cross3(e1, e2, normals + 3 * i);
        normalise3(normals + 3 * i);
    }
}

/* glibc exp (the fork's std::exp(double), :808), for checking the restatement. */
void orc_exp_batch(const double* in, double* out, uint64_t n)
{
    for (uint64_t i = 0; i < n; ++i) out[i] = exp(in[i]);
}

/* ------------------------------------------------------------------------- */
/* Image::saveTextFile, src/Image.cxx:210-235: operator<<(float) = "%.6g"     */
/* ('\t' between columns, std::endl between rows, no trailing newline).      */
/* ------------------------------------------------------------------------- */
int orc_save_text(const float* image, uint32_t width, uint32_t height, const char* path)
{
    FILE* f = fopen(path, "wb");
    if (!f) return ORC_ERR_IO;
    for (uint32_t row = 0; row < height; ++row) {
        for (uint32_t col = 0; col < width; ++col) {
            fprintf(f, "%.6g", (double)image[(size_t)row * width + col]);
            if (col < width - 1) fputc('\t', f);
        }
        if (row < height - 1) fputc('\n', f);
    }
    fclose(f);
    return ORC_OK;
}

/* std::exp(float) as the reference calls it (glibc expf). */
float orc_expf(float x) { return expf(x); }

void orc_expf_batch(const float* in, float* out, uint64_t n)
{
    for (uint64_t i = 0; i < n; ++i) out[i] = expf(in[i]);
}

uint8_t orc_lut_u8(float v) { return lut_u8(v); }

/* ------------------------------------------------------------------------- */
/* Hit pairs: every (pixel, triangle) whose Ray::intersect reports a hit with */
/* t > 1e-7 (main.cxx:683-687), for the rows of a list.  Used to test that   */
/* the GPU's conservative footprints contain every real hit.                 */
/* ------------------------------------------------------------------------- */
struct pairs_job {
    const float* tris;
    uint64_t ntris;
    const float* cam;
    uint32_t width, height;
    const uint32_t* rows;
    uint32_t nrows;
    uint32_t* out_pixel;   /* (row index in list) * width + col */
    uint32_t* out_tri;
    uint64_t cap, count;
    uint32_t next;
    pthread_mutex_t lock;
};

static void* pairs_worker(void* arg)
{
    struct pairs_job* job = (struct pairs_job*)arg;
    const float* cam = job->cam;
    for (;;) {
        pthread_mutex_lock(&job->lock);
        uint32_t i = job->next++;
        pthread_mutex_unlock(&job->lock);
        if (i >= job->nrows) break;
        uint32_t row = job->rows[i];
        for (uint32_t col = 0; col < job->width; ++col) {
            float v_offset = (float)((double)cam[12] * (0.5 + (double)row - (double)job->height / 2.0));
            float u_offset = (float)((double)cam[12] * (0.5 + (double)col - (double)job->width / 2.0));
            float dir[3];
            for (int k = 0; k < 3; ++k)
                dir[k] = ((cam[3 + k] + cam[6 + k] * v_offset) + cam[9 + k] * u_offset) - cam[k];
            normalise3(dir);
            float d[3] = {0.0f, 0.0f, 0.0f};
            float len = length3(dir);
            if (fpclassify(len) != FP_ZERO) {
                d[0] = dir[0] / len;
                d[1] = dir[1] / len;
                d[2] = dir[2] / len;
            }
            for (uint64_t j = 0; j < job->ntris; ++j) {
                const float* tr = job->tris + 9 * j;
                float t;
                if (orc_intersect(cam, d, tr, tr + 3, tr + 6, &t) && (double)t > 0.0000001) {
                    pthread_mutex_lock(&job->lock);
                    if (job->count < job->cap) {
                        job->out_pixel[job->count] = i * job->width + col;
                        job->out_tri[job->count] = (uint32_t)j;
                    }
                    ++job->count;
                    pthread_mutex_unlock(&job->lock);
                }
            }
        }
    }
    return NULL;
}

int64_t orc_hit_pairs(const float* tris, uint64_t ntris, const float cam[13], uint32_t width,
                      uint32_t height, const uint32_t* rows, uint32_t nrows, uint32_t* out_pixel,
                      uint32_t* out_tri, uint64_t cap, int nthreads)
{
    struct pairs_job job;
    memset(&job, 0, sizeof job);
    job.tris = tris;
    job.ntris = ntris;
    job.cam = cam;
    job.width = width;
    job.height = height;
    job.rows = rows;
    job.nrows = nrows;
    job.out_pixel = out_pixel;
    job.out_tri = out_tri;
    job.cap = cap;
    pthread_mutex_init(&job.lock, NULL);
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    for (int i = 1; i < nthreads; ++i) pthread_create(&th[i], NULL, pairs_worker, &job);
    pairs_worker(&job);
    for (int i = 1; i < nthreads; ++i) pthread_join(th[i], NULL);
    pthread_mutex_destroy(&job.lock);
    return (int64_t)job.count;
}
