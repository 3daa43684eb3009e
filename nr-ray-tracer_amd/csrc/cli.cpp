// `nrt-cli render <scene>` — host driver mirroring the reference's `render`
// command (packages/ray-tracer/src/commands/render.rs:104-115, cli.rs:111-270):
// same flags and NR_RT_CAMERA_* environment variables, render timed alone
// (render.rs:57-62), gamma 0.5 + to_rgb8 + write (render.rs:74-102).
// Extra flags: --precision {f64,f32}, --rng {chacha8,philox}, --gpus N, --legacy-schema (also
// load the index schema of scenes/triangles.toml, NRT_LOAD_LEGACY_SCHEMA).
// Output formats: .png (stored deflate), .ppm, .pfm (linear f32).
//
// `nrt-cli convert-stl <STL> [-o FILE] [-f] [-F toml|json]` — the reference's
// `create convert-stl` (app/commands/create/convert_stl.rs:19-138): binary STL
// -> one Group of Triangles, vertices read as (x, z, -y), k = 1 / max extent,
// point = k (a - p_min), u = k (b - a), v = k (c - a), camera look_at
// (k l/2, k h/2, 0), look_from = look_at + Z, white background, fov 50,
// 50 bounces, spp 200, "# model bbox" header line.
#include <array>
#include <charconv>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <regex>
#include <string>
#include <thread>
#include <vector>

#include "nrt.h"

namespace {

[[noreturn]] void die(const std::string& m) {
    fprintf(stderr, "Error: %s\n", m.c_str());
    exit(1);
}

bool parse_vec(const std::string& s, double out[3]) {  // cli.rs:71-90  "^(\S+),(\S+),(\S+)$"
    static const std::regex re(R"(^\s*(\S+),(\S+),(\S+)\s*$)");
    std::smatch m;
    if (!std::regex_match(s, m, re)) return false;
    for (int k = 0; k < 3; ++k) {
        char* end = nullptr;
        std::string t = m[k + 1].str();
        out[k] = strtod(t.c_str(), &end);
        if (t.empty() || *end) return false;
    }
    return true;
}

bool parse_ratio(const std::string& s, double& r) {  // cli.rs:92-109
    char* end = nullptr;
    r = strtod(s.c_str(), &end);
    if (!s.empty() && *end == '\0') return true;
    static const std::regex re(R"(^\s*(\d+)\s*/\s*(\d+)\s*$)");
    std::smatch m;
    if (!std::regex_match(s, m, re)) return false;
    r = strtod(m[1].str().c_str(), nullptr) / strtod(m[2].str().c_str(), nullptr);
    return true;
}

uint32_t crc_table[256];
void crc_init() {
    for (uint32_t n = 0; n < 256; ++n) {
        uint32_t c = n;
        for (int k = 0; k < 8; ++k) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
        crc_table[n] = c;
    }
}
uint32_t crc(const uint8_t* p, size_t n, uint32_t c = 0xFFFFFFFFu) {
    for (size_t k = 0; k < n; ++k) c = crc_table[(c ^ p[k]) & 0xFF] ^ (c >> 8);
    return c;
}

void be32(std::vector<uint8_t>& v, uint32_t x) {
    v.push_back(x >> 24); v.push_back(x >> 16); v.push_back(x >> 8); v.push_back(x);
}

void chunk(FILE* f, const char* type, const std::vector<uint8_t>& data) {
    std::vector<uint8_t> c;
    be32(c, (uint32_t)data.size());
    c.insert(c.end(), type, type + 4);
    c.insert(c.end(), data.begin(), data.end());
    const uint32_t cr = crc(c.data() + 4, c.size() - 4) ^ 0xFFFFFFFFu;
    be32(c, cr);
    fwrite(c.data(), 1, c.size(), f);
}

void write_png(FILE* f, uint32_t w, uint32_t h, const std::vector<uint8_t>& rgb) {
    crc_init();
    static const uint8_t sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
    fwrite(sig, 1, 8, f);
    std::vector<uint8_t> ihdr;
    be32(ihdr, w);
    be32(ihdr, h);
    ihdr.insert(ihdr.end(), {8, 2, 0, 0, 0});
    chunk(f, "IHDR", ihdr);
    std::vector<uint8_t> raw;
    for (uint32_t y = 0; y < h; ++y) {
        raw.push_back(0);
        raw.insert(raw.end(), rgb.begin() + (size_t)y * w * 3, rgb.begin() + (size_t)(y + 1) * w * 3);
    }
    std::vector<uint8_t> z = {0x78, 0x01};
    uint32_t a = 1, b = 0;
    for (uint8_t x : raw) { a = (a + x) % 65521; b = (b + a) % 65521; }
    size_t pos = 0;
    do {
        const size_t n = std::min<size_t>(65535, raw.size() - pos);
        z.push_back(pos + n == raw.size() ? 1 : 0);
        z.push_back(n & 0xFF); z.push_back(n >> 8);
        z.push_back(~n & 0xFF); z.push_back((~n >> 8) & 0xFF);
        z.insert(z.end(), raw.begin() + (long)pos, raw.begin() + (long)(pos + n));
        pos += n;
    } while (pos < raw.size());
    be32(z, (b << 16) | a);
    chunk(f, "IDAT", z);
    chunk(f, "IEND", {});
}

std::string shortest(double x) {  // Rust's f64 Display: shortest round-trip digits, "1.0" style
    if (x == 0.0) return std::signbit(x) ? "-0.0" : "0.0";
    char buf[64];
    auto r = std::to_chars(buf, buf + sizeof buf, x);
    std::string t(buf, r.ptr);
    if (t.find_first_of(".eEn") == std::string::npos) t += ".0";
    return t;
}

int convert_stl(int argc, char** argv) {  // argv[1] == "convert-stl"
    std::string input, output, format = "toml";
    bool force = false;
    for (int i = 2; i < argc; ++i) {
        const std::string a = argv[i];
        auto val = [&]() -> std::string {
            if (i + 1 >= argc) die("missing value for " + a);
            return argv[++i];
        };
        if (a == "-o" || a == "--output") output = val();
        else if (a == "-f" || a == "--force-overwrite") force = true;
        else if (a == "-F" || a == "--format") format = val();
        else if (!a.empty() && a[0] == '-') die("unknown option " + a);
        else input = a;
    }
    if (input.empty()) die("missing STL file");
    if (format != "toml" && format != "json") die("--format must be toml or json");
    FILE* in = fopen(input.c_str(), "rb");
    if (!in) die("No such file or directory (os error 2)");
    uint8_t header[80];
    uint32_t count = 0;
    if (fread(header, 1, 80, in) != 80 || fread(&count, 4, 1, in) != 1) die("failed to fill whole buffer");
    using V = std::array<double, 3>;
    std::vector<std::array<V, 3>> tris(count);
    V lo{INFINITY, INFINITY, INFINITY}, hi{-INFINITY, -INFINITY, -INFINITY};
    for (uint32_t t = 0; t < count; ++t) {
        float f[12];
        uint16_t attr;
        if (fread(f, 4, 12, in) != 12 || fread(&attr, 2, 1, in) != 1) die("failed to fill whole buffer");
        for (int k = 0; k < 3; ++k) {  // skip the normal (f[0..2]); DVec3::new(x, z, -y)
            const V p{(double)f[3 + 3 * k], (double)f[5 + 3 * k], -(double)f[4 + 3 * k]};
            tris[t][k] = p;
            for (int r = 0; r < 3; ++r) { lo[r] = std::min(lo[r], p[r]); hi[r] = std::max(hi[r], p[r]); }
        }
    }
    fclose(in);
    const double l = hi[0] - lo[0], h = hi[1] - lo[1], w = hi[2] - lo[2];
    const double k = 1.0 / std::max(std::max(l, w), h);
    const V look_at{k * l / 2.0, k * h / 2.0, 0.0};
    const V look_from{look_at[0], look_at[1], look_at[2] + 1.0};
    auto vec = [](const V& v) { return "[" + shortest(v[0]) + ", " + shortest(v[1]) + ", " + shortest(v[2]) + "]"; };
    std::string out;
    char hdr[128];
    snprintf(hdr, sizeof hdr, "# model bbox: l=%.4f h=%.4f w=%.4f\n", k * l, k * h, k * w);
    out += hdr;
    std::vector<std::array<V, 3>> puv;
    for (auto& t : tris) {
        V p, u, v;
        for (int r = 0; r < 3; ++r) {
            p[r] = k * (t[0][r] - lo[r]);
            u[r] = k * (t[1][r] - t[0][r]);
            v[r] = k * (t[2][r] - t[0][r]);
        }
        puv.push_back({p, u, v});
    }
    if (format == "toml") {
        out += "[camera]\nbackground_color = [1.0, 1.0, 1.0]\nlook_at = " + vec(look_at) + "\nlook_from = " + vec(look_from) +
               "\nfield_of_view = 50.0\nsamples_per_pixel = 200\nray_max_bounces = 50\n\n[[scene]]\n\n[scene.Group]\n";
        for (auto& t : puv)
            out += "\n[[scene.Group.objects]]\n\n[scene.Group.objects.Triangle]\npoint = " + vec(t[0]) + "\nu = " + vec(t[1]) +
                   "\nv = " + vec(t[2]) + "\n";
    } else {
        out += "{\n  \"camera\": {\n    \"width\": null,\n    \"height\": null,\n    \"aspect_ratio\": null,\n"
               "    \"background_color\": [1.0, 1.0, 1.0],\n    \"look_at\": " + vec(look_at) + ",\n    \"look_from\": " +
               vec(look_from) + ",\n    \"view_up\": null,\n    \"focal_length\": null,\n    \"field_of_view\": 50.0,\n"
               "    \"defocus_angle\": null,\n    \"focus_distance\": null,\n    \"samples_per_pixel\": 200,\n"
               "    \"ray_max_bounces\": 50\n  },\n  \"scene\": [\n    {\n      \"Group\": {\n        \"objects\": [";
        for (size_t i = 0; i < puv.size(); ++i)
            out += std::string(i ? "," : "") + "\n          {\"Triangle\": {\"point\": " + vec(puv[i][0]) + ", \"u\": " +
                   vec(puv[i][1]) + ", \"v\": " + vec(puv[i][2]) + "}}";
        out += "\n        ]\n      }\n    }\n  ]\n}";
    }
    if (output.empty()) {
        fwrite(out.data(), 1, out.size(), stdout);
        return 0;
    }
    if (!force) {
        if (FILE* e = fopen(output.c_str(), "rb")) { fclose(e); die("File exists (os error 17)"); }
    }
    FILE* o = fopen(output.c_str(), "wb");
    if (!o) die("cannot open " + output);
    fwrite(out.data(), 1, out.size(), o);
    fclose(o);
    return 0;
}

void usage() {
    fprintf(stderr,
            "usage: nrt-cli convert-stl <STL> [-o FILE] [-f] [-F toml|json]\n"
            "       nrt-cli render <SCENE> [-o FILE] [-f] [--gamma-value G] [-W W] [-H H] [--aspect-ratio R]\n"
            "       [--background-color X,Y,Z] [--look-at X,Y,Z] [--look-from X,Y,Z] [--view-up X,Y,Z]\n"
            "       [--focal-length F] [--field-of-view DEG] [--defocus-angle DEG] [--focus-distance D]\n"
            "       [--samples-per-pixel N] [--ray-max-bounces N] [-v]\n"
            "       [--precision f64|f32] [--rng chacha8|philox] [--gpus N] [--legacy-schema]\n");
    exit(2);
}

}  // namespace

int main(int argc, char** argv) {
    if (argc >= 3 && std::string(argv[1]) == "convert-stl") return convert_stl(argc, argv);
    if (argc < 3 || std::string(argv[1]) != "render") usage();
    std::string scene, output = "out.png";
    bool force = false, verbose = false;
    uint32_t load_flags = 0;
    float gamma = 0.5f;
    int gpus = 1;
    nrt_camera_config cc{};
    nrt_render_opts opts{};
    opts.device = -1;

    // environment first, then flags (clap: flag value beats env)
    struct EnvKey { const char* env; const char* flag; };
    static const EnvKey envs[] = {
        {"NR_RT_CAMERA_WIDTH", "--width"}, {"NR_RT_CAMERA_HEIGHT", "--height"},
        {"NR_RT_CAMERA_ASPECT_RATIO", "--aspect-ratio"}, {"NR_RT_CAMERA_BACKGROUND_COLOR", "--background-color"},
        {"NR_RT_CAMERA_LOOK_AT", "--look-at"}, {"NR_RT_CAMERA_LOOK_FROM", "--look-from"},
        {"NR_RT_CAMERA_VIEW_UP", "--view-up"}, {"NR_RT_CAMERA_FOCAL_LENGTH", "--focal-length"},
        {"NR_RT_CAMERA_FIELD_OF_VIEW", "--field-of-view"}, {"NR_RT_CAMERA_DEFOCUS_ANGLE", "--defocus-angle"},
        {"NR_RT_CAMERA_FOCUS_DISTANCE", "--focus-distance"},
        {"NR_RT_CAMERA_SAMPLES_PER_PIXEL", "--samples-per-pixel"},
        {"NR_RT_CAMERA_RAY_MAX_BOUNCES", "--ray-max-bounces"}};
    std::vector<std::pair<std::string, std::string>> kv;
    for (const auto& e : envs)
        if (const char* v = getenv(e.env)) kv.emplace_back(e.flag, v);
    for (int i = 2; i < argc; ++i) {
        std::string a = argv[i];
        auto val = [&]() -> std::string {
            if (i + 1 >= argc) die("missing value for " + a);
            return argv[++i];
        };
        if (a == "-o" || a == "--output") output = val();
        else if (a == "-f" || a == "--force-overwrite") force = true;
        else if (a == "-v" || a == "--verbose") verbose = true;
        else if (a == "--gamma-value") gamma = strtof(val().c_str(), nullptr);
        else if (a == "-W") kv.emplace_back("--width", val());
        else if (a == "-H") kv.emplace_back("--height", val());
        else if (a == "--precision") {
            std::string p = val();
            opts.precision = p == "f32" ? NRT_PRECISION_F32 : p == "f64" ? NRT_PRECISION_F64 : 99;
            if (opts.precision == 99) die("--precision must be f64 or f32");
        } else if (a == "--rng") {
            std::string r = val();
            opts.rng = r == "philox" ? NRT_RNG_PHILOX : r == "chacha8" ? NRT_RNG_CHACHA8 : 99;
            if (opts.rng == 99) die("--rng must be chacha8 or philox");
        } else if (a == "--gpus") gpus = atoi(val().c_str());
        else if (a == "--legacy-schema") load_flags |= NRT_LOAD_LEGACY_SCHEMA;  // a switch: takes no value
        else if (a.rfind("--", 0) == 0) kv.emplace_back(a, val());
        else if (scene.empty()) scene = a;
        else usage();
    }
    if (scene.empty()) usage();
    for (auto& kvp : kv) {
        const std::string& k = kvp.first;
        const std::string& v = kvp.second;
        double d3[3];
        char* end = nullptr;
        auto u64 = [&]() { uint64_t x = strtoull(v.c_str(), &end, 10); if (*end) die("invalid value '" + v + "' for " + k); return x; };
        auto f64 = [&]() { double x = strtod(v.c_str(), &end); if (*end) die("invalid value '" + v + "' for " + k); return x; };
        auto vec = [&](double* dst, uint32_t bit) { if (!parse_vec(v, d3)) die("Invalid vector: '" + v + "'"); memcpy(dst, d3, sizeof d3); cc.set |= bit; };
        if (k == "--width") { cc.width = u64(); cc.set |= NRT_CC_WIDTH; }
        else if (k == "--height") { cc.height = u64(); cc.set |= NRT_CC_HEIGHT; }
        else if (k == "--aspect-ratio") { if (!parse_ratio(v, cc.aspect_ratio)) die("Invalid image ratio: '" + v + "'"); cc.set |= NRT_CC_ASPECT_RATIO; }
        else if (k == "--background-color") vec(cc.background_color, NRT_CC_BACKGROUND_COLOR);
        else if (k == "--look-at") vec(cc.look_at, NRT_CC_LOOK_AT);
        else if (k == "--look-from") vec(cc.look_from, NRT_CC_LOOK_FROM);
        else if (k == "--view-up") vec(cc.view_up, NRT_CC_VIEW_UP);
        else if (k == "--focal-length") { cc.focal_length = f64(); cc.set |= NRT_CC_FOCAL_LENGTH; }
        else if (k == "--field-of-view") { cc.field_of_view = f64(); cc.set |= NRT_CC_FIELD_OF_VIEW; }
        else if (k == "--defocus-angle") { cc.defocus_angle = f64(); cc.set |= NRT_CC_DEFOCUS_ANGLE; }
        else if (k == "--focus-distance") { cc.focus_distance = f64(); cc.set |= NRT_CC_FOCUS_DISTANCE; }
        else if (k == "--samples-per-pixel") { cc.samples_per_pixel = u64(); cc.set |= NRT_CC_SAMPLES_PER_PIXEL; }
        else if (k == "--ray-max-bounces") { cc.ray_max_bounces = u64(); cc.set |= NRT_CC_RAY_MAX_BOUNCES; }
        else die("unknown flag " + k);
    }

    // ImageConfig::get_file (cli.rs:140-154): decide format and open before rendering
    const size_t dot = output.find_last_of('.');
    const std::string ext = dot == std::string::npos ? "" : output.substr(dot + 1);
    if (ext != "png" && ext != "ppm" && ext != "pfm") die("The image format could not be determined");
    if (!force) {
        if (FILE* f = fopen(output.c_str(), "rb")) { fclose(f); die("File exists (os error 17)"); }
    }
    FILE* out = fopen(output.c_str(), "wb");
    if (!out) die("cannot open " + output);

    nrt_scene* sc = nullptr;
    nrt_camera cam{};
    if (nrt_scene_load_ex(scene.c_str(), &cc, load_flags, &sc, &cam) != NRT_OK) die(nrt_last_error());
    const uint32_t W = (uint32_t)cam.width, H = (uint32_t)cam.height;
    std::vector<float> img((size_t)W * H * 3);

    // GPU runtime start, the scene's upload and (--gpus N > 1) the multi-GPU context before the timed
    // render (render.rs:57-62 times scene.render alone; the scene was built before it), reported apart
    // with -v
    const auto ti = std::chrono::steady_clock::now();
    int ndev = nrt_device_count();
    if (gpus < 1) gpus = 1;
    // (tests: NRT_MULTI_LOOPBACK=1 puts the N shards on device 0, csrc/multi.hip; NRT_CLI_SHARDS=1 takes the
    // per-device row-shard threads below, as without RCCL)
    const char* lb = getenv("NRT_MULTI_LOOPBACK");
    const bool loopback = lb && *lb && strcmp(lb, "0") != 0;
    const char* fs = getenv("NRT_CLI_SHARDS");
    const bool force_shards = fs && strcmp(fs, "1") == 0;
    if (gpus > ndev && !loopback) die("requested " + std::to_string(gpus) + " GPUs, " + std::to_string(ndev) + " visible");
    auto dev_of = [&](int g) { return loopback ? 0 : g; };
    // --gpus N > 1: the library's multi-GPU render (nrt_render_opts.gpus): rows interleaved over
    // devices 0 .. N-1, one RCCL gather to device 0, un-permuted there; without a usable
    // librccl (nrt_render_prepare: NRT_E_UNSUPPORTED) one host thread per device renders its row shard
    // and the frame is un-permuted here
    bool shards = false;
    if (gpus > 1) {
        opts.gpus = (uint32_t)gpus;
        const int rc = force_shards ? NRT_E_UNSUPPORTED : nrt_render_prepare(sc, &cam, &opts);
        if (rc == NRT_E_UNSUPPORTED) {
            if (verbose) fprintf(stderr, " multi-GPU render without RCCL (%s): per-device row shards\n", nrt_last_error());
            opts.gpus = 0;
            shards = true;
            for (int g = 0; g < gpus; ++g)
                if (nrt_scene_upload(sc, dev_of(g)) != NRT_OK) die(nrt_last_error());
        } else if (rc != NRT_OK) {
            die(nrt_last_error());
        }
    } else if (nrt_render_prepare(sc, &cam, &opts) != NRT_OK) {
        die(nrt_last_error());
    }
    const double init_secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - ti).count();
    const auto t0 = std::chrono::steady_clock::now();
    if (shards) {
        std::vector<std::vector<float>> part((size_t)gpus);
        std::vector<std::string> err((size_t)gpus);
        std::vector<std::thread> th;
        for (int g = 0; g < gpus; ++g)
            th.emplace_back([&, g]() {
                nrt_render_opts o = opts;
                o.device = dev_of(g);
                o.row_offset = (uint32_t)g;
                o.row_stride = (uint32_t)gpus;
                part[(size_t)g].resize((size_t)nrt_rows_selected(H, &o) * W * 3);
                if (nrt_render(sc, &cam, &o, part[(size_t)g].data(), part[(size_t)g].size(), nullptr, nullptr) != NRT_OK)
                    err[(size_t)g] = nrt_last_error();
            });
        for (auto& t : th) t.join();
        for (const auto& e : err)
            if (!e.empty()) die(e);
        for (uint32_t y = 0; y < H; ++y)  // frame row y = shard y % N, its row y / N
            memcpy(&img[(size_t)y * W * 3], &part[y % (uint32_t)gpus][(size_t)(y / (uint32_t)gpus) * W * 3],
                   (size_t)W * 3 * sizeof(float));
    } else if (nrt_render(sc, &cam, &opts, img.data(), img.size(), nullptr, nullptr) != NRT_OK) {
        die(nrt_last_error());
    }
    const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (verbose) {
        const double samples = (double)W * H * (double)cam.samples_per_pixel;
        fprintf(stderr, " GPU runtime start + scene upload: %.3f secs\n", init_secs);
        fprintf(stderr, " Rendering - Done in %.3f secs (%.1f Msamples/s)\n", secs, samples / secs / 1e6);
    }

    if (ext == "pfm") {
        fprintf(out, "PF\n%u %u\n-1.0\n", W, H);
        for (uint32_t y = H; y-- > 0;) fwrite(&img[(size_t)y * W * 3], sizeof(float), (size_t)W * 3, out);
    } else {
        std::vector<uint8_t> rgb(img.size());
        nrt_image_to_rgb8(img.data(), img.size(), gamma, rgb.data());
        if (ext == "ppm") {
            fprintf(out, "P6\n%u %u\n255\n", W, H);
            fwrite(rgb.data(), 1, rgb.size(), out);
        } else {
            write_png(out, W, H, rgb);
        }
    }
    fclose(out);
    nrt_scene_destroy(sc);
    return 0;
}
