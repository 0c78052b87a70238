// halogen_render — a native host driving the path through the C++ HalogenRenderPass (include/halogen_render_pass.hpp).
//
//   halogen_render render SCENE.hgscene CONFIG.txt OUT.f32 [device]   progressive frames, writes RGBA32F rows
//   halogen_render params CONFIG.txt                                    prints make_params' bytes as hex (no GPU)
//
// SCENE.hgscene: "HGSCENE1", int32 counts of spheres, meshes, materials, triangles, BVH entries, then the arrays in
// the reference's struct layouts (44/164/84/72/32 B) — what UpdateObjectBuffers uploads (RP:448-509).
// CONFIG.txt: one "key value..." per line: the HalogenSettings fields by their reference names, the camera
// (width, height, fov, position x y z, rotation x y z w, localToWorld 16 floats in Unity field order), frames, and optionally
// cubemap PATH ("HGCUBE01", int32 face size, int32 mips, int64 float count, floats).  halogen/host_files.py writes
// all three from the Python scene description.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iostream>
#include <map>
#include <sstream>
#include <string>
#include <vector>

#include "halogen_render_pass.hpp"

namespace {

struct Config {
    halogen::HalogenSettings settings;
    halogen::Camera camera;
    int32_t frames = 1, frame_count = 1, n_spheres = 0, n_meshes = 0;
    std::string cubemap_path;
};

[[noreturn]] void die(const std::string& msg) {
    std::fprintf(stderr, "halogen_render: %s\n", msg.c_str());
    std::exit(2);
}

Config read_config(const std::string& path) {
    std::ifstream in(path);
    if (!in) die("cannot open " + path);
    Config c;
    halogen::HalogenSettings& s = c.settings;
    std::string line;
    while (std::getline(in, line)) {
        std::istringstream ls(line);
        std::string k;
        if (!(ls >> k) || k[0] == '#') continue;
        auto f = [&]() {
            std::string v;
            if (!(ls >> v)) die("missing value for " + k);
            return std::strtof(v.c_str(), nullptr);  // nearest float, as Python's float32 conversion
        };
        auto i = [&]() {
            long v;
            if (!(ls >> v)) die("missing value for " + k);
            return int32_t(v);
        };
        if (k == "width") c.camera.pixelWidth = i();
        else if (k == "height") c.camera.pixelHeight = i();
        else if (k == "fov") c.camera.fieldOfView = f();
        else if (k == "position") { c.camera.position.x = f(); c.camera.position.y = f(); c.camera.position.z = f(); }
        else if (k == "rotation") {
            c.camera.rotation.x = f(); c.camera.rotation.y = f(); c.camera.rotation.z = f(); c.camera.rotation.w = f();
        }
        else if (k == "localToWorld") { for (float& m : c.camera.localToWorld.m) m = f(); }
        else if (k == "frames") c.frames = i();
        else if (k == "frame_count") c.frame_count = i();
        else if (k == "n_spheres") c.n_spheres = i();
        else if (k == "n_meshes") c.n_meshes = i();
        else if (k == "cubemap") { if (!(ls >> c.cubemap_path)) die("missing cubemap path"); }
        else if (k == "ShowInSceneView") s.ShowInSceneView = i() != 0;
        else if (k == "Accumulate") s.Accumulate = i() != 0;
        else if (k == "SamplesPerPixel") s.SamplesPerPixel = i();
        else if (k == "MaxAccumulatedFrames") s.MaxAccumulatedFrames = i();
        else if (k == "UnlimitedSampling") s.UnlimitedSampling = i() != 0;
        else if (k == "MaxBounces") s.MaxBounces = i();
        else if (k == "DiffuseBounces") s.DiffuseBounces = i();
        else if (k == "GlossyBounces") s.GlossyBounces = i();
        else if (k == "TransmissionBounces") s.TransmissionBounces = i();
        else if (k == "FilterRadius") s.FilterRadius = f();
        else if (k == "NearPlaneDistance") s.NearPlaneDistance = f();
        else if (k == "FarPlaneDistance") s.FarPlaneDistance = f();
        else if (k == "FocalPlaneDistance") s.FocalPlaneDistance = f();
        else if (k == "ApertureAngle") s.ApertureAngle = f();
        else if (k == "useHDRISky") s.useHDRISky = i() != 0;
        else if (k == "EnvironmentMipLevel") s.EnvironmentMipLevel = i();
        else if (k == "FirstInteractionOnly") s.FirstInteractionOnly = i() != 0;
        else if (k == "DebugMode") s.DebugMode = halogen::HalogenDebugMode(i());
        else if (k == "TriangleDebugDisplayRange") s.TriangleDebugDisplayRange = i();
        else if (k == "BoxDebugDisplayRange") s.BoxDebugDisplayRange = i();
        else die("unknown key " + k);
    }
    return c;
}

template <class T>
void read_array(std::ifstream& in, std::vector<T>& v, int32_t n, const char* what) {
    if (n < 0) die(std::string("negative count of ") + what);
    v.resize(size_t(n));
    if (n && !in.read(reinterpret_cast<char*>(v.data()), std::streamsize(sizeof(T) * size_t(n))))
        die(std::string("short read of ") + what);
}

halogen::SceneBuffers read_scene(const std::string& path) {
    std::ifstream in(path, std::ios::binary);
    if (!in) die("cannot open " + path);
    char magic[8];
    int32_t n[5];
    if (!in.read(magic, 8) || std::string(magic, 8) != "HGSCENE1") die(path + ": not an HGSCENE1 file");
    if (!in.read(reinterpret_cast<char*>(n), sizeof(n))) die(path + ": short header");
    halogen::SceneBuffers sc;
    read_array(in, sc.spheres, n[0], "spheres");
    read_array(in, sc.meshes, n[1], "meshes");
    read_array(in, sc.materials, n[2], "materials");
    read_array(in, sc.triangles, n[3], "triangles");
    read_array(in, sc.blas, n[4], "BVH entries");
    return sc;
}

halogen::Cubemap read_cubemap(const std::string& path) {
    std::ifstream in(path, std::ios::binary);
    if (!in) die("cannot open " + path);
    char magic[8];
    int32_t fm[2];
    int64_t nf = 0;
    if (!in.read(magic, 8) || std::string(magic, 8) != "HGCUBE01") die(path + ": not an HGCUBE01 file");
    if (!in.read(reinterpret_cast<char*>(fm), sizeof(fm)) || !in.read(reinterpret_cast<char*>(&nf), sizeof(nf)))
        die(path + ": short header");
    halogen::Cubemap c;
    c.face_size = fm[0];
    c.n_mips = fm[1];
    c.texels.resize(size_t(nf));
    if (nf && !in.read(reinterpret_cast<char*>(c.texels.data()), std::streamsize(sizeof(float) * size_t(nf))))
        die(path + ": short read");
    return c;
}

}  // namespace

int main(int argc, char** argv) {
    const std::string mode = argc > 1 ? argv[1] : "";
    if (mode == "params" && argc == 3) {
        const Config c = read_config(argv[2]);
        halogen::Cubemap dummy;
        halogen::HalogenSettings st = c.settings;
        if (!c.cubemap_path.empty()) st.environmentCubemap = &dummy;  // only its presence matters here
        const halogen::ClampedSettings s = halogen::clamp_settings(st);
        const hg_params p = halogen::make_params(s, c.camera, c.frame_count, c.n_spheres, c.n_meshes,
                                                 s.UseEnvironmentCubemap);
        const unsigned char* b = reinterpret_cast<const unsigned char*>(&p);
        for (size_t k = 0; k < sizeof(p); ++k) std::printf("%02x", b[k]);
        std::printf("\n");
        return 0;
    }
    if (mode == "display" && (argc == 6 || argc == 7)) {  // one Execute per frame with the pipelined display
        const halogen::SceneBuffers scene = read_scene(argv[2]);
        Config c = read_config(argv[3]);
        halogen::Cubemap cube;
        if (!c.cubemap_path.empty()) {
            cube = read_cubemap(c.cubemap_path);
            c.settings.environmentCubemap = &cube;
        }
        const std::string fmt_name = argv[5];
        const int32_t fmt = fmt_name == "rgba32f" ? HG_DISPLAY_RGBA32F : fmt_name == "rgba16f" ? HG_DISPLAY_RGBA16F
                            : fmt_name == "r11g11b10f" ? HG_DISPLAY_R11G11B10F : -1;
        if (fmt < 0) die("display format must be rgba32f, rgba16f or r11g11b10f");
        try {
            halogen::HalogenRenderPass pass(c.settings, argc == 7 ? std::atoi(argv[6]) : 0);
            pass.SetDisplay(fmt, 1);  // one frame behind, as the C# pass
            int shown = 0;
            const auto t0 = std::chrono::steady_clock::now();
            for (int32_t f = 0; f < c.frames; ++f) {
                pass.Execute(scene, c.camera, 1);
                if (pass.Display().data) ++shown;
            }
            const halogen::HalogenRenderPass::DisplayImage last = pass.FlushDisplay();
            const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
            if (!last.data) die("no image displayed");
            std::ofstream out(argv[4], std::ios::binary);
            out.write(static_cast<const char*>(last.data), std::streamsize(last.bytes));
            if (!out) die(std::string("cannot write ") + argv[4]);
            std::printf("{\"frames\": %d, \"shown_while_rendering\": %d, \"frame_count\": %d, \"format\": %d, "
                        "\"bytes\": %zu, \"ms_per_frame\": %.4f}\n",
                        c.frames, shown, pass.getFrameCount(), last.format, last.bytes, ms / std::max(1, c.frames));
        } catch (const halogen::HalogenError& e) {
            std::fprintf(stderr, "halogen_render: %s\n", e.what());
            return 1;
        }
        return 0;
    }
    if (mode != "render" || argc < 5 || argc > 6) {
        std::fprintf(stderr,
                     "usage: %s render SCENE.hgscene CONFIG.txt OUT.f32 [device]\n"
                     "       %s display SCENE.hgscene CONFIG.txt OUT.bin rgba32f|rgba16f|r11g11b10f [device]\n"
                     "       %s params CONFIG.txt\n",
                     argv[0], argv[0], argv[0]);
        return 2;
    }
    const halogen::SceneBuffers scene = read_scene(argv[2]);
    Config c = read_config(argv[3]);
    halogen::Cubemap cube;
    if (!c.cubemap_path.empty()) {
        cube = read_cubemap(c.cubemap_path);
        c.settings.environmentCubemap = &cube;
    }
    try {
        halogen::HalogenRenderPass pass(c.settings, argc == 6 ? std::atoi(argv[5]) : 0);
        pass.SetCounters(true);  // (printed below)
        pass.Execute(scene, c.camera, c.frames);
        const std::vector<float> img = pass.Readback();
        const hg_counters cnt = pass.Counters();
        std::ofstream out(argv[4], std::ios::binary);
        out.write(reinterpret_cast<const char*>(img.data()), std::streamsize(img.size() * sizeof(float)));
        if (!out) die(std::string("cannot write ") + argv[4]);
        std::printf("{\"frames\": %d, \"frame_count\": %d, \"paths\": %llu, \"rays\": %llu, \"tri_tests\": %llu, "
                    "\"aabb_tests\": %llu}\n",
                    c.frames, pass.getFrameCount(), (unsigned long long)cnt.paths, (unsigned long long)cnt.rays,
                    (unsigned long long)cnt.tri_tests, (unsigned long long)cnt.aabb_tests);
    } catch (const halogen::HalogenError& e) {
        std::fprintf(stderr, "halogen_render: %s\n", e.what());
        return 1;
    }
    return 0;
}
