// dcrt_render -- a C++ host of the MI355X wavefront path tracer in the shape of the reference's
// application: CScene + the CPathTracer plugin slot filled by CMI355XPathTracer
// (mi355x_path_tracer.h, the C ABI of include/dcrt.h alone) and the reference's frame loop
// (renderer_loop.h: LoadScene, DispatchRayTracing with its small-resolution first frame and
// frame-seed policies, SampleConvolution of each completed image), then "Save Image to File".
//
//   dcrt_render <scene.obj|scene.xml> <width> <height> <spp> <max_bounce> <out.bmp>
//               [--batch] [--point x y z r g b] [--seed-type sample-count|frame-index|fixed]
//               [--fixed-seed N] [--iterations N] [--pool N] [--film out.f32] [--samples out.f32]
//
// Frame-loop mode (default) runs frames until `spp` full-resolution images are in the film;
// --batch instead hands all images to dcrt_tracer_render_images (device-side image
// sequencing). --film writes the raw RGBA32F film (sum w*L, sum w), --samples the last image's
// sample textures (positions W*H*2 then values W*H*4 floats). The last stdout line is JSON.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "dcrt.h"
#include "mi355x_path_tracer.h"
#include "renderer_loop.h"

namespace {

bool Check(int rc, const char* what)
{
    if (rc == DCRT_OK) return true;
    std::fprintf(stderr, "%s failed (%d): %s\n", what, rc, dcrt_last_error());
    return false;
}

bool WriteFloats(const char* path, const std::vector<float>& a, const std::vector<float>* b = nullptr)
{
    FILE* f = std::fopen(path, "wb");
    if (!f) return false;
    bool ok = std::fwrite(a.data(), sizeof(float), a.size(), f) == a.size();
    if (ok && b) ok = std::fwrite(b->data(), sizeof(float), b->size(), f) == b->size();
    return std::fclose(f) == 0 && ok;
}

int Usage(const char* exe)
{
    std::fprintf(stderr,
                 "usage: %s scene.{obj,xml} width height spp max_bounce out.bmp [--batch] [--point x y z r g b]\n"
                 "       [--seed-type sample-count|frame-index|fixed] [--fixed-seed N] [--iterations N] [--pool N]\n"
                 "       [--film out.f32] [--samples out.f32]\n",
                 exe);
    return 2;
}

}  // namespace

int main(int argc, char** argv)
{
    if (argc < 7) return Usage(argv[0]);
    const char* scenePath = argv[1];
    const uint32_t width = (uint32_t)std::atoi(argv[2]), height = (uint32_t)std::atoi(argv[3]);
    const uint32_t spp = (uint32_t)std::atoi(argv[4]), maxBounce = (uint32_t)std::atoi(argv[5]);
    const char* outPath = argv[6];
    bool batch = false, pointLight = false;
    float lightPos[3] = {0, 0, 0}, lightColor[3] = {0, 0, 0};
    CRendererLoop::EFrameSeedType seedType = CRendererLoop::EFrameSeedType::SampleCount;
    uint32_t fixedSeed = 0, iterations = 16, pool = 0;
    const char* filmPath = nullptr;
    const char* samplesPath = nullptr;
    for (int i = 7; i < argc; ++i) {
        const bool more = i + 1 < argc;
        if (!std::strcmp(argv[i], "--batch")) {
            batch = true;
        } else if (!std::strcmp(argv[i], "--point") && i + 6 < argc) {
            pointLight = true;
            for (int k = 0; k < 3; ++k) lightPos[k] = (float)std::atof(argv[i + 1 + k]);
            for (int k = 0; k < 3; ++k) lightColor[k] = (float)std::atof(argv[i + 4 + k]);
            i += 6;
        } else if (!std::strcmp(argv[i], "--seed-type") && more) {
            const std::string v = argv[++i];
            if (v == "sample-count") seedType = CRendererLoop::EFrameSeedType::SampleCount;
            else if (v == "frame-index") seedType = CRendererLoop::EFrameSeedType::FrameIndex;
            else if (v == "fixed") seedType = CRendererLoop::EFrameSeedType::Fixed;
            else return Usage(argv[0]);
        } else if (!std::strcmp(argv[i], "--fixed-seed") && more) {
            fixedSeed = (uint32_t)std::atoi(argv[++i]);
        } else if (!std::strcmp(argv[i], "--iterations") && more) {
            iterations = (uint32_t)std::atoi(argv[++i]);
        } else if (!std::strcmp(argv[i], "--pool") && more) {
            pool = (uint32_t)std::atoi(argv[++i]);
        } else if (!std::strcmp(argv[i], "--film") && more) {
            filmPath = argv[++i];
        } else if (!std::strcmp(argv[i], "--samples") && more) {
            samplesPath = argv[++i];
        } else {
            return Usage(argv[0]);
        }
    }
    if (width == 0 || height == 0 || spp == 0 || iterations == 0) return Usage(argv[0]);

    // CDirectComputeRayTracing::Init: new + Create (LaunchRendererLoop.cpp:58-64)
    CScene scene;
    CMI355XPathTracer tracer(pool ? pool : (batch ? (1u << 24) : (1u << 21)), iterations);
    CRendererLoop loop(&scene, &tracer);
    loop.m_FrameSeedType = seedType;
    if (!scene.m_Handle) return 1;
    if (!tracer.Create()) return 1;

    // LoadScene: Reset + LoadFromFile (+ UI "Create -> Point Light", max bounce), then
    // OnSceneLoaded and the small-resolution size
    scene.m_IsFilmDirty = true;
    if (!scene.Reset(width, height) || !scene.LoadFromFile(scenePath)) {
        std::fprintf(stderr, "LoadScene failed: %s\n", dcrt_last_error());
        return 1;
    }
    if (pointLight) {
        const float euler[3] = {0, 0, 0};
        if (!Check(dcrt_scene_add_punctual_light(scene.m_Handle, lightPos, euler, lightColor, 0), "AddPointLight")) return 1;
    }
    if (!Check(dcrt_scene_set_max_bounce(scene.m_Handle, maxBounce), "SetMaxBounce")) return 1;
    if (!loop.AfterSceneEdited()) return 1;
    if (seedType == CRendererLoop::EFrameSeedType::Fixed) scene.m_FrameSeed = fixedSeed;   // the UI's seed field (ImGui.cpp:157-160)

    const auto t0 = std::chrono::steady_clock::now();
    uint32_t firstSeed = 0;
    uint64_t previewFrames = 0;
    std::vector<uint32_t> seeds;   // frame seed of each full-resolution image, in film order
    if (batch) {
        const dcrt_filter_params filter = MakeFilter(scene);
        if (!Check(dcrt_tracer_clear_film(tracer.GetTracer()), "ClearFilm") ||
            !Check(dcrt_tracer_render_images(tracer.GetTracer(), 0, spp, &filter), "RenderImages"))
            return 1;
        for (uint32_t s = 0; s < spp; ++s) seeds.push_back(s);
    } else {
        // RenderOneFrame until spp full-resolution images are in the film
        const uint64_t maxFrames = (uint64_t)spp * 100000ull + 1000ull;
        while (seeds.size() < spp) {
            SRenderContext rc;
            if (!loop.RenderOneFrame(&rc)) return 1;
            if (rc.m_IsSmallResolutionEnabled) {
                ++previewFrames;
                continue;
            }
            // (the seed advances right after the image completes, except under Fixed)
            if (loop.m_LastFrameCompletedImage)
                seeds.push_back(seedType == CRendererLoop::EFrameSeedType::Fixed ? scene.m_FrameSeed : scene.m_FrameSeed - 1u);
            if (loop.m_FrameIndex > maxFrames) {
                std::fprintf(stderr, "the frame loop did not complete %u images\n", spp);
                return 1;
            }
        }
        firstSeed = seeds.empty() ? 0 : seeds.front();
    }
    if (!Check(dcrt_tracer_synchronize(tracer.GetTracer()), "Synchronize")) return 1;
    const double seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();

    const uint32_t W = scene.m_ResolutionWidth, H = scene.m_ResolutionHeight;   // (an XML scene sets its own)
    const size_t n = (size_t)W * H;
    if (filmPath) {
        std::vector<float> film(n * 4);
        if (!Check(dcrt_tracer_read_film(tracer.GetTracer(), film.data()), "ReadFilm") || !WriteFloats(filmPath, film)) return 1;
    }
    if (samplesPath) {
        std::vector<float> pos(n * 2), val(n * 4);
        if (!Check(dcrt_tracer_read_samples(tracer.GetTracer(), pos.data(), val.data()), "ReadSamples") ||
            !WriteFloats(samplesPath, pos, &val))
            return 1;
    }
    // post-processing + "Save Image to File"
    dcrt_postfx_params post;
    if (!Check(dcrt_scene_get_postfx_params(scene.m_Handle, &post), "GetPostFxParams")) return 1;
    std::vector<uint8_t> rgba(n * 4);
    float sumLogLuminance = 0.0f;
    if (!Check(dcrt_tracer_resolve_image(tracer.GetTracer(), &post, rgba.data(), &sumLogLuminance), "ResolveImage")) return 1;
    if (!Check(dcrt_write_bmp(outPath, W, H, rgba.data()), "WriteBmp")) return 1;
    dcrt_ray_stats stats;
    if (!Check(dcrt_tracer_counters(tracer.GetTracer(), &stats), "Counters")) return 1;
    const double rays = (double)(stats.extension_rays + stats.shadow_rays);
    std::string seedList;
    for (size_t i = 0; i < seeds.size(); ++i) seedList += (i ? "," : "") + std::to_string(seeds[i]);
    std::printf("{\"images\": %u, \"seconds\": %.4f, \"ms_per_spp\": %.3f, \"mrays_per_s\": %.1f, \"extension_rays\": %llu, "
                "\"shadow_rays\": %llu, \"mode\": \"%s\", \"frames\": %llu, \"preview_frames\": %llu, \"first_seed\": %u, "
                "\"seeds\": [%s]}\n",
                spp, seconds, seconds * 1e3 / spp, rays / seconds / 1e6, (unsigned long long)stats.extension_rays,
                (unsigned long long)stats.shadow_rays, batch ? "render_images" : "frame_loop", (unsigned long long)loop.m_FrameIndex,
                (unsigned long long)previewFrames, firstSeed, seedList.c_str());
    return 0;
}
