// main.cpp -- xrt_main: the reference's command line (src/main.cxx:182-392)
// over the MI355X render path.
//
//   -h, --help                 usage
//   -s, --size W H             image size (default 2048 2048)
//   -b, --background R G B     parsed and unused, as in the reference
//   -f, --filename NAME        output text file "./out/NAME" (default test.jpg,
//                              which, as in the reference, receives text)
//   -i, --input FILE           mesh file (default ./dragon.ply); repeatable: the
//                              files' meshes make one scene, in order
// additions:
//   -g, --gpus N               row strips over N GPUs (default 1)
//   -k, --kernel brute|tiled|binned  render kernel (default: automatic -- tiled
//                              for small frames, binned past 2e7 footprint tests)
//   -t, --threads N            accepted for main-pthreads*.cxx compatibility (ignored)
//       --signed               the L-buffer fork (main-pthreads-lbuffer.cxx): signed
//                              multi-material L-buffer + hole fill
//       --lbuffer FILE         also write the L-buffer as raw little-endian f32
//       --u8 FILE              also write the 8-bit image (LUT 0..80) as PGM
//       --time                 print render wall-clock and Mrays/s
//       --rows A:B             render image rows [A, B) only and write that
//                              strip (B - A text rows), as one pthreads
//                              thread's share of the frame
//       --batch N              render the frame N times back to back (one
//                              xrt_render_frames call) and write the last;
//                              with --time, the device time per frame
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <iostream>
#include <stdexcept>
#include <string>
#include <vector>

#include "Image.h"
#include "RayTracer.h"
#include "TriangleMesh.h"
#include "xrt.h"

namespace {

void showUsage(const std::string& prog)
{
    std::cerr << "Usage: " << prog << " <option(s)>\n"
              << "Options:\n"
              << "\t-h,--help\t\t\tShow this help message\n"
              << "\t-s,--size IMG_WIDTH IMG_HEIGHT\tSpecify the image size in number of pixels (default values: 2048 2048)\n"
              << "\t-b,--background R G B\t\tSpecify the background colour in RGB (accepted, unused)\n"
              << "\t-f,--filename FILENAME\t\tName of the output text file, written to ./out/ (default: test.jpg)\n"
              << "\t-i,--input FILENAME\t\tInput mesh, PLY or OBJ (default: ./dragon.ply); repeat for a scene of several files\n"
              << "\t-g,--gpus N\t\t\tRender row strips on N GPUs (default: 1)\n"
              << "\t-k,--kernel brute|tiled|binned\tRender kernel (default: automatic)\n"
              << "\t--signed\t\t\tSigned multi-material L-buffer and hole fill (main-pthreads-lbuffer.cxx)\n"
              << "\t--lbuffer FILE\t\t\tWrite the L-buffer as raw float32\n"
              << "\t--u8 FILE\t\t\tWrite the 8-bit image (0..80 keV LUT) as PGM\n"
              << "\t--time\t\t\t\tPrint render time and Mrays/s\n"
              << "\t--rows A:B\t\t\tRender and write image rows [A, B) only\n"
              << "\t--batch N\t\t\tRender the frame N times back to back, write the last\n"
              << std::endl;
}

struct Options {
    std::string output = "test.jpg";
    std::vector<std::string> inputs;
    unsigned width = 2048, height = 2048;
    int gpus = 1;
    int kernel = XRT_KERNEL_AUTO;
    std::string lbuffer, u8;
    bool time = false;
    bool signed_model = false;
    bool rows = false;
    unsigned row_begin = 0, row_end = 0;
    unsigned batch = 0;
};

unsigned parse_uint(const char* prog, int argc, char** argv, int& i)
{
    if (++i >= argc) {
        showUsage(prog);
        std::exit(EXIT_FAILURE);
    }
    return (unsigned)std::stoi(argv[i]);
}

std::string parse_str(const char* prog, int argc, char** argv, int& i)
{
    if (++i >= argc) {
        showUsage(prog);
        std::exit(EXIT_FAILURE);
    }
    return argv[i];
}

Options processCmd(int argc, char** argv)
{
    Options o;
    for (int i = 1; i < argc; ++i) {
        std::string a = argv[i];
        if (a == "-h" || a == "--help") {
            showUsage(argv[0]);
            std::exit(EXIT_SUCCESS);
        } else if (a == "-s" || a == "--size") {
            o.width = parse_uint(argv[0], argc, argv, i);
            o.height = parse_uint(argv[0], argc, argv, i);
        } else if (a == "-b" || a == "--background") {
            for (int k = 0; k < 3; ++k) (void)parse_uint(argv[0], argc, argv, i);
        } else if (a == "-f" || a == "--filename") {
            o.output = "./out/" + parse_str(argv[0], argc, argv, i);
        } else if (a == "-i" || a == "--input") {
            o.inputs.push_back(parse_str(argv[0], argc, argv, i));
        } else if (a == "-g" || a == "--gpus") {
            o.gpus = (int)parse_uint(argv[0], argc, argv, i);
        } else if (a == "-t" || a == "--threads") {
            (void)parse_uint(argv[0], argc, argv, i);
        } else if (a == "-k" || a == "--kernel") {
            std::string k = parse_str(argv[0], argc, argv, i);
            if (k == "brute") o.kernel = XRT_KERNEL_BRUTE;
            else if (k == "tiled") o.kernel = XRT_KERNEL_TILED;
            else if (k == "binned") o.kernel = XRT_KERNEL_BINNED;
            else {
                showUsage(argv[0]);
                std::exit(EXIT_FAILURE);
            }
        } else if (a == "--lbuffer") {
            o.lbuffer = parse_str(argv[0], argc, argv, i);
        } else if (a == "--u8") {
            o.u8 = parse_str(argv[0], argc, argv, i);
        } else if (a == "--signed") {
            o.signed_model = true;
        } else if (a == "--time") {
            o.time = true;
        } else if (a == "--rows") {
            const std::string r = parse_str(argv[0], argc, argv, i);
            const size_t colon = r.find(':');
            if (colon == std::string::npos || colon == 0 || colon + 1 >= r.size()) {
                showUsage(argv[0]);
                std::exit(EXIT_FAILURE);
            }
            o.rows = true;
            o.row_begin = (unsigned)std::stoul(r.substr(0, colon));
            o.row_end = (unsigned)std::stoul(r.substr(colon + 1));
        } else if (a == "--batch") {
            o.batch = parse_uint(argv[0], argc, argv, i);
            if (!o.batch) {
                showUsage(argv[0]);
                std::exit(EXIT_FAILURE);
            }
        } else {
            showUsage(argv[0]);
            std::exit(EXIT_FAILURE);
        }
    }
    if (o.inputs.empty()) o.inputs.push_back("./dragon.ply");
    if (o.rows && (o.row_begin >= o.row_end || o.row_end > o.height))
        throw std::out_of_range("--rows A:B must satisfy 0 <= A < B <= image height");
    if ((o.rows || o.batch) && (o.signed_model || o.gpus > 1))
        throw std::runtime_error("--rows and --batch render the attenuation model on one GPU");
    return o;
}

}  // namespace

int main(int argc, char** argv)
{
    try {
        Options opt = processCmd(argc, argv);
        setRenderKernel(opt.kernel);

        std::cout << "Loading polygon meshes... " << std::endl;
        auto t0 = std::chrono::high_resolution_clock::now();
        std::vector<TriangleMesh> meshes;
        loadMeshes(opt.inputs[0], meshes);
        for (size_t f = 1; f < opt.inputs.size(); ++f) appendMeshes(opt.inputs[f], meshes);
        auto t1 = std::chrono::high_resolution_clock::now();
        std::cout << "Loading meshes took: " << std::chrono::duration<double>(t1 - t0).count()
                  << " seconds" << std::endl
                  << std::endl;

        std::cout << "Getting scene bbox... " << std::endl;
        Vec3 lower, upper;
        getBBox(meshes, upper, lower);
        float lut = 0.0f;
        Image image(opt.width, opt.height, lut);
        RayTracerInfo info = initialiseRayTracing(meshes, upper, lower, opt.height, opt.width, image, lut);

        auto r0 = std::chrono::high_resolution_clock::now();
        std::vector<float> lb;
        const unsigned rb = opt.rows ? opt.row_begin : 0u, re = opt.rows ? opt.row_end : opt.height;
        double ms_per_frame = 0.0;
        if (opt.batch) {                          // N frames back to back, the last one kept
            xrt_stats st;
            ms_per_frame = renderLoopFrames(image, meshes, info, opt.batch, rb, re, &st);
            for (unsigned long long k = 0; k < st.odd_rays; ++k) std::cout << "Only one intersect on this ray" << std::endl;
        } else if (opt.rows && opt.lbuffer.empty()) {
            xrt_stats st;
            renderLoopRows(image, meshes, info, rb, re, nullptr, nullptr, &st);
            for (unsigned long long k = 0; k < st.odd_rays; ++k) std::cout << "Only one intersect on this ray" << std::endl;
        } else if (opt.signed_model && opt.gpus > 1) {
            renderLoopLBufferMultiGPU(image, meshes, info, opt.gpus, opt.lbuffer.empty() ? nullptr : &lb);
        } else if (opt.signed_model) {
            renderLoopLBuffer(image, meshes, info, opt.lbuffer.empty() ? nullptr : &lb);
        } else if (opt.gpus > 1) {
            renderLoopMultiGPU(image, meshes, info, opt.gpus);
        } else if (!opt.lbuffer.empty()) {       // the image and the L-buffer in one render
            lb.resize((size_t)opt.width * (re - rb));
            xrt_stats st;
            renderLoopRows(image, meshes, info, rb, re, lb.data(), nullptr, &st);
            for (unsigned long long k = 0; k < st.odd_rays; ++k) std::cout << "Only one intersect on this ray" << std::endl;
        } else {
            renderLoop(image, meshes, info);
        }
        auto r1 = std::chrono::high_resolution_clock::now();
        if (opt.time) {
            double s = std::chrono::duration<double>(r1 - r0).count();
            const double rays = (double)opt.width * (re - rb);
            std::cout << "Render took: " << s << " seconds (" << rays * (opt.batch ? opt.batch : 1) / s / 1e6
                      << " Mrays/s, " << opt.gpus << " GPU(s))" << std::endl;
            if (opt.batch)
                std::cout << "Frames: " << opt.batch << ", device time per frame " << ms_per_frame << " ms ("
                          << rays / (ms_per_frame * 1e3) << " Mrays/s)" << std::endl;
        }

        Image* out = &image;
        Image strip;
        if (opt.rows) {                           // the strip's rows only
            strip = Image(opt.width, re - rb, 0.0f);
            std::copy(image.getData() + (size_t)rb * opt.width, image.getData() + (size_t)re * opt.width,
                      strip.getData());
            out = &strip;
        }
        out->saveTextFile(opt.output);
        if (!opt.u8.empty()) out->savePGMFile(opt.u8, 0.0f, 80.0f);
        if (!opt.lbuffer.empty()) {
            if (lb.empty()) {                   // multi-GPU, batch: the L-buffer of the same frame
                lb.resize((size_t)opt.width * (re - rb));
                xrt_stats st;
                renderLoopRows(image, meshes, info, rb, re, lb.data(), nullptr, &st);
            }
            std::FILE* f = std::fopen(opt.lbuffer.c_str(), "wb");
            if (!f) throw std::runtime_error("Cannot create the file " + opt.lbuffer);
            std::fwrite(lb.data(), sizeof(float), lb.size(), f);
            std::fclose(f);
        }
    } catch (const std::exception& e) {
        std::cerr << "ERROR: " << e.what() << std::endl;
        return 1;
    } catch (const std::string& e) {
        std::cerr << "ERROR: " << e << std::endl;
        return 2;
    } catch (const char* e) {
        std::cerr << "ERROR: " << e << std::endl;
        return 3;
    }
    return 0;
}
