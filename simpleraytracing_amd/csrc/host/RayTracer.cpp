// RayTracer.cpp -- see RayTracer.h.
#include "RayTracer.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <limits>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <thread>

#include "PlyLoader.h"
#include "xrt.h"
#include "xrt_host.h"

namespace {

int g_kernel = -1;
int g_device = -1;

int kernel_choice()
{
    if (g_kernel >= 0) return g_kernel;
    const char* k = std::getenv("XRT_KERNEL");
    if (k && std::strcmp(k, "brute") == 0) return XRT_KERNEL_BRUTE;
    if (k && std::strcmp(k, "tiled") == 0) return XRT_KERNEL_TILED;
    if (k && std::strcmp(k, "binned") == 0) return XRT_KERNEL_BINNED;
    return XRT_KERNEL_AUTO;
}

int device_choice()
{
    if (g_device >= 0) return g_device;
    const char* d = std::getenv("XRT_DEVICE");
    return d ? std::atoi(d) : 0;
}

void check(xrt_context* ctx, int rc, const char* what)
{
    if (rc != XRT_OK)
        throw std::runtime_error(std::string(what) + ": " + xrt_last_error(ctx));
}

}  // namespace

// One context per device for the process lifetime (contexts are not
// thread-safe, so each is guarded by its own mutex).  Contexts are released by
// process exit, not by static destructors that could run after the HIP
// runtime has been torn down.
struct DeviceSlot {
    std::mutex lock;
    xrt_context* ctx = nullptr;
    std::vector<float> mesh;   // the soup last uploaded (renders of the same mesh skip the upload)
    bool uploaded = false;
};

static DeviceSlot& device_slot(int device)
{
    static std::mutex registry_lock;
    static std::map<int, std::unique_ptr<DeviceSlot>> slots;
    std::lock_guard<std::mutex> g(registry_lock);
    auto& slot = slots[device];
    if (!slot) slot.reset(new DeviceSlot());
    if (!slot->ctx) {
        xrt_context* ctx = nullptr;
        int rc = xrt_create(device, &ctx);
        if (rc != XRT_OK) throw std::runtime_error(std::string("xrt_create: ") + xrt_last_error(nullptr));
        slot->ctx = ctx;
    }
    return *slot;
}

xrt_context* xrt_host_device_context(int device) { return device_slot(device).ctx; }

void setRenderKernel(int kernel) { g_kernel = kernel; }
void setRenderDevice(int device) { g_device = device; }

// Assimp-free loadMeshes (main.cxx:455-508): each mesh of the file through
// TriangleMesh::setGeometry(vertices, indices), in file order.
void appendMeshes(const std::string& file_name, std::vector<TriangleMesh>& meshes)
{
    const std::string ext = file_name.size() >= 4 ? file_name.substr(file_name.size() - 4) : "";
    std::vector<PlyMesh> parts;
    if (ext == ".obj" || ext == ".OBJ") parts = loadObj(file_name);
    else parts.push_back(loadPly(file_name));
    for (const PlyMesh& part : parts) {
        TriangleMesh mesh;
        mesh.setGeometry(part.vertices, part.indices);
        meshes.push_back(mesh);
    }
}

void loadMeshes(const std::string& file_name, std::vector<TriangleMesh>& meshes)
{
    std::vector<TriangleMesh> loaded;
    appendMeshes(file_name, loaded);
    meshes.swap(loaded);
}

// main.cxx:538-563
void getBBox(const std::vector<TriangleMesh>& meshes, Vec3& upper, Vec3& lower)
{
    const float inf = std::numeric_limits<float>::infinity();
    lower = Vec3(inf, inf, inf);
    upper = Vec3(-inf, -inf, -inf);
    for (const TriangleMesh& m : meshes) {
        for (unsigned k = 0; k < 3; ++k) {
            lower[k] = std::min(lower[k], m.getLowerBBoxCorner()[k]);
            upper[k] = std::max(upper[k], m.getUpperBBoxCorner()[k]);
        }
    }
}

// main.cxx:566-622; the arithmetic is xrt_camera_from_bbox's.
RayTracerInfo initialiseRayTracing(std::vector<TriangleMesh>&, const Vec3& upper, const Vec3& lower,
                                   unsigned int image_height, unsigned int image_width,
                                   Image& output_image, float lut)
{
    float lo[3] = {lower[0], lower[1], lower[2]};
    float hi[3] = {upper[0], upper[1], upper[2]};
    xrt_camera cam;
    if (xrt_camera_from_bbox(lo, hi, image_width, image_height, &cam) != XRT_OK)
        throw std::runtime_error("initialiseRayTracing: invalid image size or bounding box");
    output_image = Image(image_width, image_height, lut);
    RayTracerInfo info;
    info.detector_position = Vec3(cam.detector[0], cam.detector[1], cam.detector[2]);
    info.origin = Vec3(cam.origin[0], cam.origin[1], cam.origin[2]);
    info.up = Vec3(cam.up[0], cam.up[1], cam.up[2]);
    info.right = Vec3(cam.right[0], cam.right[1], cam.right[2]);
    // main.cxx:598-601: a white light at the source, pointing at the box centre
    const Vec3 range = upper - lower;
    Vec3 light_direction = (lower + range / 2.0) - info.origin;
    light_direction.normalise();
    info.light = Light(Vec3(1.0f, 1.0f, 1.0f), light_direction, info.origin);
    info.upper_bbox_corner = upper;
    info.lower_bbox_corner = lower;
    info.range = range;
    return info;
}

namespace {

// Camera for a render: RayTracerInfo + the pixel spacing of renderLoop's
// prologue (main.cxx:634-641), from the bbox of all meshes.
xrt_camera camera_for(const Image& image, const std::vector<TriangleMesh>& meshes,
                      const RayTracerInfo& info)
{
    Vec3 upper, lower;
    getBBox(meshes, upper, lower);
    Vec3 range = upper - lower;
    float res1 = range[2] / image.getWidth();
    float res2 = range[1] / image.getHeight();
    xrt_camera cam;
    for (unsigned k = 0; k < 3; ++k) {
        cam.origin[k] = info.origin[k];
        cam.detector[k] = info.detector_position[k];
        cam.up[k] = info.up[k];
        cam.right[k] = info.right[k];
    }
    cam.pixel_spacing = 2 * std::max(res1, res2);
    cam.width = image.getWidth();
    cam.height = image.getHeight();
    return cam;
}

void render_strip(int device, const xrt_camera& cam, const std::vector<float>& soup,
                  unsigned row_begin, unsigned row_end, float* image_strip, float* lbuffer_strip,
                  unsigned char* u8_strip, xrt_stats* stats)
{
    DeviceSlot& slot = device_slot(device);
    std::lock_guard<std::mutex> g(slot.lock);
    xrt_context* ctx = slot.ctx;
    check(ctx, xrt_set_kernel(ctx, kernel_choice()), "xrt_set_kernel");
    if (!slot.uploaded || slot.mesh != soup) {   // the mesh lives on the device between renders
        check(ctx, xrt_upload_mesh(ctx, soup.data(), soup.size() / 9), "xrt_upload_mesh");
        slot.mesh = soup;
        slot.uploaded = true;
    }
    check(ctx, xrt_render_rows(ctx, &cam, row_begin, row_end, image_strip, lbuffer_strip, u8_strip, stats),
          "xrt_render_rows");
}

std::vector<float> mesh0_soup(const std::vector<TriangleMesh>& meshes)
{
    // Only hits on meshes[0] count (main.cxx:687); other meshes cannot change
    // the image, so only mesh 0 is sent to the device.
    return meshes.empty() ? std::vector<float>() : meshes[0].flatten();
}

void report_odd(unsigned long long odd)
{
    for (unsigned long long i = 0; i < odd; ++i) std::cout << "Only one intersect on this ray" << std::endl;
}

}  // namespace

void renderLoopRows(Image& image, const std::vector<TriangleMesh>& meshes, const RayTracerInfo& info,
                    unsigned int row_begin, unsigned int row_end, float* lbuffer_strip,
                    unsigned char* u8_strip, xrt_stats* stats)
{
    if (row_begin > row_end || row_end > image.getHeight())
        throw std::out_of_range("renderLoopRows: row range outside the image");
    xrt_camera cam = camera_for(image, meshes, info);
    std::vector<float> soup = mesh0_soup(meshes);
    render_strip(device_choice(), cam, soup, row_begin, row_end,
                 image.getData() + (size_t)row_begin * image.getWidth(), lbuffer_strip, u8_strip, stats);
}

double renderLoopFrames(Image& image, const std::vector<TriangleMesh>& meshes, const RayTracerInfo& info,
                        unsigned int frames, unsigned int row_begin, unsigned int row_end, xrt_stats* stats)
{
    if (row_begin > row_end || row_end > image.getHeight())
        throw std::out_of_range("renderLoopFrames: row range outside the image");
    xrt_camera cam = camera_for(image, meshes, info);
    std::vector<float> soup = mesh0_soup(meshes);
    DeviceSlot& slot = device_slot(device_choice());
    std::lock_guard<std::mutex> g(slot.lock);
    xrt_context* ctx = slot.ctx;
    check(ctx, xrt_set_kernel(ctx, kernel_choice()), "xrt_set_kernel");
    if (!slot.uploaded || slot.mesh != soup) {
        check(ctx, xrt_upload_mesh(ctx, soup.data(), soup.size() / 9), "xrt_upload_mesh");
        slot.mesh = soup;
        slot.uploaded = true;
    }
    double ms = 0.0;
    check(ctx, xrt_render_frames(ctx, &cam, row_begin, row_end, frames,
                                 image.getData() + (size_t)row_begin * image.getWidth(), nullptr, nullptr, stats, &ms),
          "xrt_render_frames");
    return ms;
}

namespace {
thread_local unsigned long long t_last_odd_rays = 0;
}

void renderLoop(Image& image, const std::vector<TriangleMesh>& meshes, RayTracerInfo& info)
{
    xrt_stats stats;
    renderLoopRows(image, meshes, info, 0, image.getHeight(), nullptr, nullptr, &stats);
    report_odd(stats.odd_rays);
    t_last_odd_rays = stats.odd_rays;
}

unsigned long long renderLoopOddRays() { return t_last_odd_rays; }

unsigned long long renderLoopLBuffer(Image& image, const std::vector<TriangleMesh>& meshes, RayTracerInfo& info,
                                     std::vector<float>* lbuffer)
{
    xrt_camera cam = camera_for(image, meshes, info);
    std::vector<float> soup = mesh0_soup(meshes);
    DeviceSlot& slot = device_slot(device_choice());
    std::lock_guard<std::mutex> g(slot.lock);
    xrt_context* ctx = slot.ctx;
    int k = kernel_choice();
    check(ctx, xrt_set_kernel(ctx, k == XRT_KERNEL_TILED ? XRT_KERNEL_BINNED : k), "xrt_set_kernel");
    if (!slot.uploaded || slot.mesh != soup) {
        check(ctx, xrt_upload_mesh(ctx, soup.data(), soup.size() / 9), "xrt_upload_mesh");
        slot.mesh = soup;
        slot.uploaded = true;
    }
    check(ctx, xrt_set_model(ctx, XRT_MODEL_SIGNED, 0.1037f), "xrt_set_model");   // :800
    if (lbuffer) lbuffer->resize((size_t)image.getWidth() * image.getHeight());
    xrt_stats stats;
    const int rc = xrt_render_signed(ctx, &cam, image.getData(), lbuffer ? lbuffer->data() : nullptr, nullptr, &stats);
    xrt_set_model(ctx, XRT_MODEL_ATTENUATION, 0.0f);
    check(ctx, rc, "xrt_render_signed");
    return stats.odd_rays;
}

namespace {

// One multi-device context per device list for the process lifetime: the
// devices 0 .. num_gpus-1, or $XRT_MULTI_DEVICES ("0,0" ...; a device listed
// twice rehearses the strip path on one GPU).  Guarded by multi_lock().
std::mutex& multi_lock()
{
    static std::mutex lock;
    return lock;
}

xrt_multi* multi_context(int num_gpus)
{
    std::vector<int> devices;
    if (const char* env = std::getenv("XRT_MULTI_DEVICES")) {
        std::string list(env);
        for (size_t pos = 0; pos < list.size();) {
            size_t next = list.find(',', pos);
            if (next == std::string::npos) next = list.size();
            devices.push_back(std::atoi(list.substr(pos, next - pos).c_str()));
            pos = next + 1;
        }
    } else {
        int available = xrt_device_count();
        if (num_gpus < 1 || num_gpus > available)
            throw std::runtime_error("renderLoopMultiGPU: " + std::to_string(num_gpus) + " GPUs requested, " +
                                     std::to_string(available) + " available");
        for (int g = 0; g < num_gpus; ++g) devices.push_back(g);
    }
    static std::map<std::vector<int>, xrt_multi*> contexts;
    xrt_multi*& m = contexts[devices];
    if (!m && xrt_multi_create(devices.data(), (int)devices.size(), &m) != XRT_OK) {
        m = nullptr;
        throw std::runtime_error(std::string("xrt_multi_create: ") + xrt_multi_last_error(nullptr));
    }
    return m;
}

void mcheck(xrt_multi* m, int rc, const char* what)
{
    if (rc != XRT_OK) throw std::runtime_error(std::string(what) + ": " + xrt_multi_last_error(m));
}

}  // namespace

// Row strips over num_gpus devices gathered into device 0 with RCCL
// (xrt_render_rows_multi).
unsigned long long renderLoopMultiGPU(Image& image, const std::vector<TriangleMesh>& meshes,
                                      RayTracerInfo& info, int num_gpus)
{
    xrt_camera cam = camera_for(image, meshes, info);
    std::vector<float> soup = mesh0_soup(meshes);
    std::lock_guard<std::mutex> g(multi_lock());
    xrt_multi* m = multi_context(num_gpus);
    mcheck(m, xrt_multi_set_model(m, XRT_MODEL_ATTENUATION, 0.0f), "xrt_multi_set_model");
    mcheck(m, xrt_multi_set_kernel(m, kernel_choice()), "xrt_multi_set_kernel");
    mcheck(m, xrt_multi_upload_mesh(m, soup.data(), soup.size() / 9), "xrt_multi_upload_mesh");
    xrt_stats stats;
    mcheck(m, xrt_render_rows_multi(m, &cam, image.getData(), nullptr, nullptr, &stats), "xrt_render_rows_multi");
    report_odd(stats.odd_rays);
    return stats.odd_rays;
}

unsigned long long renderLoopLBufferMultiGPU(Image& image, const std::vector<TriangleMesh>& meshes,
                                             RayTracerInfo& info, int num_gpus, std::vector<float>* lbuffer)
{
    xrt_camera cam = camera_for(image, meshes, info);
    std::vector<float> soup = mesh0_soup(meshes);
    std::lock_guard<std::mutex> g(multi_lock());
    xrt_multi* m = multi_context(num_gpus);
    const int k = kernel_choice();
    mcheck(m, xrt_multi_set_kernel(m, k == XRT_KERNEL_TILED ? XRT_KERNEL_BINNED : k), "xrt_multi_set_kernel");
    mcheck(m, xrt_multi_upload_mesh(m, soup.data(), soup.size() / 9), "xrt_multi_upload_mesh");
    mcheck(m, xrt_multi_set_model(m, XRT_MODEL_SIGNED, 0.1037f), "xrt_multi_set_model");   // :800
    if (lbuffer) lbuffer->resize((size_t)image.getWidth() * image.getHeight());
    xrt_stats stats;
    const int rc = xrt_render_rows_multi(m, &cam, image.getData(), lbuffer ? lbuffer->data() : nullptr, nullptr, &stats);
    xrt_multi_set_model(m, XRT_MODEL_ATTENUATION, 0.0f);
    mcheck(m, rc, "xrt_render_rows_multi");
    return stats.odd_rays;
}

// --- extern "C" helpers (include/xrt_host.h) --------------------------------
extern "C" int xrt_host_load_ply(const char* path, float** triangles, uint64_t* num_triangles)
{
    if (!path || !triangles || !num_triangles) return XRT_ERR_ARGUMENT;
    *triangles = nullptr;
    *num_triangles = 0;
    try {
        std::vector<TriangleMesh> meshes;
        loadMeshes(path, meshes);
        std::vector<float> soup = mesh0_soup(meshes);
        float* out = static_cast<float*>(std::malloc(sizeof(float) * (soup.size() ? soup.size() : 1)));
        if (!out) return XRT_ERR_ARGUMENT;
        std::memcpy(out, soup.data(), sizeof(float) * soup.size());
        *triangles = out;
        *num_triangles = soup.size() / 9;
        return XRT_OK;
    } catch (const std::exception& e) {
        return std::string(e.what()).find("Cannot open") != std::string::npos ? XRT_ERR_IO : XRT_ERR_FORMAT;
    }
}

extern "C" int xrt_host_load_meshes(const char* path, float** triangles, uint64_t** mesh_triangles,
                                    uint32_t* num_meshes)
{
    if (!path || !triangles || !mesh_triangles || !num_meshes) return XRT_ERR_ARGUMENT;
    *triangles = nullptr;
    *mesh_triangles = nullptr;
    *num_meshes = 0;
    try {
        std::vector<TriangleMesh> meshes;
        loadMeshes(path, meshes);
        std::vector<float> all;
        std::vector<uint64_t> counts;
        for (const TriangleMesh& m : meshes) {
            std::vector<float> soup = m.flatten();
            all.insert(all.end(), soup.begin(), soup.end());
            counts.push_back(soup.size() / 9);
        }
        float* t = static_cast<float*>(std::malloc(sizeof(float) * (all.size() ? all.size() : 1)));
        uint64_t* c = static_cast<uint64_t*>(std::malloc(sizeof(uint64_t) * (counts.size() ? counts.size() : 1)));
        if (!t || !c) {
            std::free(t);
            std::free(c);
            return XRT_ERR_ARGUMENT;
        }
        std::memcpy(t, all.data(), sizeof(float) * all.size());
        std::memcpy(c, counts.data(), sizeof(uint64_t) * counts.size());
        *triangles = t;
        *mesh_triangles = c;
        *num_meshes = (uint32_t)counts.size();
        return XRT_OK;
    } catch (const std::exception& e) {
        return std::string(e.what()).find("Cannot open") != std::string::npos ? XRT_ERR_IO : XRT_ERR_FORMAT;
    }
}

extern "C" void xrt_host_free(void* p) { std::free(p); }
