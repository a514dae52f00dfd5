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
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <iostream>
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
        } else {
            showUsage(argv[0]);
            std::exit(EXIT_FAILURE);
        }
    }
    if (o.inputs.empty()) o.inputs.push_back("./dragon.ply");
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
        if (opt.signed_model && opt.gpus > 1) {
            renderLoopLBufferMultiGPU(image, meshes, info, opt.gpus, opt.lbuffer.empty() ? nullptr : &lb);
        } else if (opt.signed_model) {
            renderLoopLBuffer(image, meshes, info, opt.lbuffer.empty() ? nullptr : &lb);
        } else if (opt.gpus > 1) {
            renderLoopMultiGPU(image, meshes, info, opt.gpus);
        } else if (!opt.lbuffer.empty()) {       // the image and the L-buffer in one render
            lb.resize((size_t)opt.width * opt.height);
            xrt_stats st;
            renderLoopRows(image, meshes, info, 0, opt.height, lb.data(), nullptr, &st);
            for (unsigned long long k = 0; k < st.odd_rays; ++k) std::cout << "Only one intersect on this ray" << std::endl;
        } else {
            renderLoop(image, meshes, info);
        }
        auto r1 = std::chrono::high_resolution_clock::now();
        if (opt.time) {
            double s = std::chrono::duration<double>(r1 - r0).count();
            std::cout << "Render took: " << s << " seconds ("
                      << (double)opt.width * opt.height / s / 1e6 << " Mrays/s, " << opt.gpus
                      << " GPU(s))" << std::endl;
        }

        image.saveTextFile(opt.output);
        if (!opt.u8.empty()) image.savePGMFile(opt.u8, 0.0f, 80.0f);
        if (!opt.lbuffer.empty()) {
            if (lb.empty()) {                   // multi-GPU: the L-buffer of the same frame
                lb.resize((size_t)opt.width * opt.height);
                xrt_stats st;
                renderLoopRows(image, meshes, info, 0, opt.height, lb.data(), nullptr, &st);
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
