// dcrt_render -- a C++ host of the MI355X wavefront path tracer through the C ABI only
// (include/dcrt.h), in the shape of the reference's application loop
// (Source/LaunchRendererLoop.cpp): Init (Create, :58-64), LoadScene (OnSceneLoaded,
// :175), per frame DispatchRayTracing (Render + IsImageComplete + SampleConvolution with
// frame seed = image index, :203-264) and "Save Image to File" (SaveImageToFile.cpp).
//
//   dcrt_render <scene.obj|scene.xml> <width> <height> <spp> <max_bounce> <out.bmp>
//               [--batch] [--point x y z r g b]
//
// Per-frame mode (default) drives Render()/IsImageComplete() exactly like the reference's
// frame loop; --batch hands all images to dcrt_tracer_render_images (device-side image
// sequencing, image batches sharing the path pool). Both produce the same film.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "dcrt.h"

namespace {

bool Check(int rc, const char* what)
{
    if (rc == DCRT_OK) return true;
    std::fprintf(stderr, "%s failed (%d): %s\n", what, rc, dcrt_last_error());
    return false;
}

}  // namespace

int main(int argc, char** argv)
{
    if (argc < 7) {
        std::fprintf(stderr, "usage: %s scene.{obj,xml} width height spp max_bounce out.bmp [--batch] [--point x y z r g b]\n",
                     argv[0]);
        return 2;
    }
    const char* scenePath = argv[1];
    const uint32_t width = (uint32_t)std::atoi(argv[2]), height = (uint32_t)std::atoi(argv[3]);
    const uint32_t spp = (uint32_t)std::atoi(argv[4]), maxBounce = (uint32_t)std::atoi(argv[5]);
    const char* outPath = argv[6];
    bool batch = false, pointLight = false;
    float lightPos[3] = {0, 0, 0}, lightColor[3] = {0, 0, 0};
    for (int i = 7; i < argc; ++i) {
        if (!std::strcmp(argv[i], "--batch")) {
            batch = true;
        } else if (!std::strcmp(argv[i], "--point") && i + 6 < argc) {
            pointLight = true;
            for (int k = 0; k < 3; ++k) lightPos[k] = (float)std::atof(argv[i + 1 + k]);
            for (int k = 0; k < 3; ++k) lightColor[k] = (float)std::atof(argv[i + 4 + k]);
            i += 6;
        }
    }

    // CScene: Reset + LoadFromFile (+ UI "Create -> Point Light"), BVHAccel build inside
    dcrt_scene* scene = nullptr;
    if (!Check(dcrt_scene_create(&scene), "dcrt_scene_create")) return 1;
    int rc = 1;
    dcrt_tracer* tracer = nullptr;
    do {
        if (!Check(dcrt_scene_reset(scene, width, height), "Reset")) break;
        if (!Check(dcrt_scene_load_from_file(scene, scenePath), "LoadFromFile")) break;
        if (pointLight) {
            const float euler[3] = {0, 0, 0};
            if (!Check(dcrt_scene_add_punctual_light(scene, lightPos, euler, lightColor, 0), "AddPointLight")) break;
        }
        if (!Check(dcrt_scene_set_max_bounce(scene, maxBounce), "SetMaxBounce")) break;
        dcrt_flat_scene flat;
        dcrt_frame_params frame;
        dcrt_filter_params filter;
        if (!Check(dcrt_scene_get_flat(scene, &flat), "GetFlat")) break;
        if (!Check(dcrt_scene_get_frame_params(scene, 0, &frame), "GetFrameParams")) break;
        if (!Check(dcrt_scene_get_filter(scene, &filter), "GetFilter")) break;

        // CWavefrontPathTracer::Create + OnSceneLoaded
        dcrt_tracer_config cfg;
        std::memset(&cfg, 0, sizeof(cfg));
        cfg.path_pool_size = batch ? (1u << 24) : (1u << 21);
        cfg.iterations_per_render = 16;
        if (!Check(dcrt_tracer_create(&cfg, &tracer), "Create")) break;
        if (!Check(dcrt_tracer_upload_scene(tracer, &flat), "OnSceneLoaded")) break;
        if (!Check(dcrt_tracer_set_frame_params(tracer, &frame), "SetFrameParams")) break;
        if (!Check(dcrt_tracer_clear_film(tracer), "ClearFilm")) break;

        const auto t0 = std::chrono::steady_clock::now();
        bool ok = true;
        if (batch) {
            ok = Check(dcrt_tracer_render_images(tracer, 0, spp, &filter), "RenderImages");
        } else {
            // DispatchRayTracing: Render every frame; when the image completes, convolve it
            // into the film and start the next one with frame seed = image index
            for (uint32_t image = 0; ok && image < spp; ++image) {
                if (!Check(dcrt_scene_get_frame_params(scene, image, &frame), "GetFrameParams") ||
                    !Check(dcrt_tracer_set_frame_params(tracer, &frame), "SetFrameParams") ||
                    !Check(dcrt_tracer_reset_image(tracer), "ResetImage")) {
                    ok = false;
                    break;
                }
                int complete = 0;
                for (int frameIndex = 0; !complete && frameIndex < 100000; ++frameIndex) {
                    if (!Check(dcrt_tracer_render(tracer, 0), "Render") ||
                        !Check(dcrt_tracer_is_image_complete(tracer, &complete), "IsImageComplete")) {
                        ok = false;
                        break;
                    }
                }
                if (ok && !complete) {
                    std::fprintf(stderr, "image %u did not complete\n", image);
                    ok = false;
                }
                if (ok) ok = Check(dcrt_tracer_accumulate_film(tracer, &filter), "SampleConvolution");
            }
        }
        if (!ok || !Check(dcrt_tracer_synchronize(tracer), "Synchronize")) break;
        const double seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();

        // post-processing + "Save Image to File"
        dcrt_postfx_params post;
        if (!Check(dcrt_scene_get_postfx_params(scene, &post), "GetPostFxParams")) break;
        std::vector<uint8_t> rgba((size_t)width * height * 4);
        float sumLogLuminance = 0.0f;
        if (!Check(dcrt_tracer_resolve_image(tracer, &post, rgba.data(), &sumLogLuminance), "ResolveImage")) break;
        if (!Check(dcrt_write_bmp(outPath, width, height, rgba.data()), "WriteBmp")) break;
        dcrt_ray_stats stats;
        if (!Check(dcrt_tracer_counters(tracer, &stats), "Counters")) break;
        const double rays = (double)(stats.extension_rays + stats.shadow_rays);
        std::printf("{\"images\": %u, \"seconds\": %.4f, \"ms_per_spp\": %.3f, \"mrays_per_s\": %.1f, \"extension_rays\": %llu, "
                    "\"shadow_rays\": %llu, \"mode\": \"%s\"}\n",
                    spp, seconds, seconds * 1e3 / spp, rays / seconds / 1e6, (unsigned long long)stats.extension_rays,
                    (unsigned long long)stats.shadow_rays, batch ? "render_images" : "render");
        rc = 0;
    } while (false);
    if (tracer) dcrt_tracer_destroy(tracer);
    dcrt_scene_destroy(scene);
    return rc;
}
