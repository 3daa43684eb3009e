// Host-side checker for the sanitizer build (make -C nr-ray-tracer_amd sanitize).
//
// Runs every host stage the C ABI runs before a render -- the JSON / TOML readers
// and SceneConfig semantics (scene_config.cpp), the BVH build, the flattener and
// its f32 conversion (flatten.cpp, wbvh.cpp), the JPEG decoder (jpeg.cpp) and the
// canonical dump -- over each file named on the command line, under ASan + UBSan.
// Load errors are expected for malformed inputs (the library reports them as
// status codes); crashes, out-of-bounds accesses and undefined behaviour are what
// the build exists to catch.  No GPU code is linked.
//
//   host_check [--quiet] <scene.json|scene.toml|image.jpg> ...
#include <cstdio>
#include <cstring>
#include <exception>
#include <string>

#include "flatten.hpp"
#include "scene_config.hpp"

using namespace nrt;

static bool ends_with(const std::string& s, const char* suf) {
    const size_t n = std::strlen(suf);
    return s.size() >= n && s.compare(s.size() - n, n, suf) == 0;
}

int main(int argc, char** argv) {
    bool quiet = false;
    int ok = 0, rejected = 0;
    for (int i = 1; i < argc; ++i) {
        const std::string path = argv[i];
        if (path == "--quiet") { quiet = true; continue; }
        try {
            if (ends_with(path, ".jpg") || ends_with(path, ".jpeg")) {
                const DecodedImage img = decode_image_file(path);
                double sum = 0;
                for (float v : img.rgb) sum += v;
                if (!quiet) std::printf("ok   %s %ux%u sum %.6f\n", path.c_str(), img.width, img.height, sum);
            } else {
                const LoadedScene sc = load_scene_file(path, nullptr, ends_with(path, "triangles.toml"));
                const FlatScene flat = flatten_scene(sc.objects);
                const FlatScene32 f32 = to_f32(flat);
                const std::string dump = dump_graph(sc.objects);
                if (!quiet)
                    std::printf("ok   %s nodes %zu prims %zu world %zu dump %zu\n", path.c_str(), flat.nodes.size(),
                                flat.prims.size(), f32.wprims.size(), dump.size());
            }
            ++ok;
        } catch (const std::exception& e) {
            if (!quiet) std::printf("err  %s: %s\n", path.c_str(), e.what());
            ++rejected;
        }
    }
    std::printf("host_check: %d loaded, %d rejected\n", ok, rejected);
    return 0;
}
