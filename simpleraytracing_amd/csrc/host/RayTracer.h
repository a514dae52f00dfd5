// RayTracer.h -- scene set-up and the render loop of the drop-in host API.
//
// Same free functions and signatures as the reference's src/main.cxx:
//   loadMeshes           main.cxx:139-140, 427-510
//   getBBox              main.cxx:145-147, 538-563
//   initialiseRayTracing main.cxx:149-157, 566-622
//   renderLoop           main.cxx:159-161, 626-743  -> the GPU, via include/xrt.h
// plus renderLoopRows (a row strip, the pthreads twin's pixel-range idea,
// main-pthreads-redo.cxx:627-658) and renderLoopMultiGPU (row strips over
// several GPUs).  Errors surface as exceptions, as in the reference.
#pragma once

#include <string>
#include <vector>

#include "Image.h"
#include "Light.h"
#include "Material.h"
#include "TriangleMesh.h"
#include "Vec3.h"

struct xrt_stats;

// RayTracerInfo (main.cxx:111-121), member for member.
struct RayTracerInfo {
    Vec3 detector_position;
    Vec3 origin;
    Vec3 up;
    Vec3 right;
    Light light;              // initialiseRayTracing's light (main.cxx:598-601); unused by the X-ray path
    Vec3 upper_bbox_corner;
    Vec3 lower_bbox_corner;
    Vec3 range;
};

// Render options (process-wide): kernel = 0 auto, 1 brute force, 2 tiled cull,
// 3 binned cull.  Defaults come from $XRT_KERNEL ("brute" / "tiled" / "binned")
// and $XRT_DEVICE.
void setRenderKernel(int kernel);
void setRenderDevice(int device);

// Every mesh of a file, replacing `meshes` (main.cxx:455-508): a PLY file is
// one mesh, an OBJ file one mesh per object.  appendMeshes keeps the meshes
// already loaded (several input files make one scene; mesh 0 stays first).
void loadMeshes(const std::string& file_name, std::vector<TriangleMesh>& meshes);
void appendMeshes(const std::string& file_name, std::vector<TriangleMesh>& meshes);

void getBBox(const std::vector<TriangleMesh>& meshes, Vec3& upper, Vec3& lower);

RayTracerInfo initialiseRayTracing(std::vector<TriangleMesh>& meshes, const Vec3& upper,
                                   const Vec3& lower, unsigned int image_height,
                                   unsigned int image_width, Image& output_image, float lut);

// Whole image (main.cxx:159-161, the reference's declaration); prints one
// "Only one intersect on this ray" line per odd ray (main.cxx:710).
void renderLoop(Image& output_image, const std::vector<TriangleMesh>& meshes, RayTracerInfo& info);

// The number of odd rays of this thread's last renderLoop call (the lines it
// printed).
unsigned long long renderLoopOddRays();

// Rows [row_begin, row_end) of output_image only; optional L-buffer / 8-bit
// outputs of the same strip size.  Does not print.
void renderLoopRows(Image& output_image, const std::vector<TriangleMesh>& meshes,
                    const RayTracerInfo& info, unsigned int row_begin, unsigned int row_end,
                    float* lbuffer_strip, unsigned char* u8_strip, xrt_stats* stats);

// renderLoop's rows [row_begin, row_end) rendered `frames` times back to back
// (one xrt_render_frames call: every frame prepared and rendered in full, the
// host side of all of them in one pass); output_image holds the last frame,
// *stats its counters.  Returns the device time per frame in ms.  Does not print.
double renderLoopFrames(Image& output_image, const std::vector<TriangleMesh>& meshes, const RayTracerInfo& info,
                        unsigned int frames, unsigned int row_begin, unsigned int row_end, xrt_stats* stats);

// The L-buffer fork, src/main-pthreads-lbuffer.cxx: renderLoopCallBack over
// the whole image (:733-813, the signed multi-material L-buffer, mesh 0's
// coefficient 0.1037) and main's hole fill (:327-404) into output_image.
// `lbuffer` (optional) receives the fork's L_buffer (-1 flags).  Returns the
// number of flagged pixels.
unsigned long long renderLoopLBuffer(Image& output_image, const std::vector<TriangleMesh>& meshes,
                                     RayTracerInfo& info, std::vector<float>* lbuffer = nullptr);

// The same as row strips over `num_gpus` devices (the L-buffer strips gathered
// to device 0, which fills the holes of the assembled frame).
unsigned long long renderLoopLBufferMultiGPU(Image& output_image, const std::vector<TriangleMesh>& meshes,
                                             RayTracerInfo& info, int num_gpus, std::vector<float>* lbuffer = nullptr);

// Row strips over `num_gpus` devices (rows_per = H / n, remainder to the first
// strips), one host thread per device; returns the number of odd rays.
unsigned long long renderLoopMultiGPU(Image& output_image, const std::vector<TriangleMesh>& meshes,
                                      RayTracerInfo& info, int num_gpus);
