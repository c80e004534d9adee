// mi355x_path_tracer.cpp -- CMI355XPathTracer: the reference's CPathTracer slot over libdcrt.so.
// See mi355x_path_tracer.h for what is restated from the reference and why.
#include "mi355x_path_tracer.h"

#include <cstdio>
#include <cstring>

// ---- CScene ------------------------------------------------------------------------------
CScene::CScene() { (void)dcrt_scene_create(&m_Handle); }

CScene::~CScene()
{
    if (m_Handle) dcrt_scene_destroy(m_Handle);
}

bool CScene::Reset(uint32_t width, uint32_t height)
{
    if (!m_Handle || dcrt_scene_reset(m_Handle, width, height) != DCRT_OK) return false;
    m_ResolutionWidth = width;
    m_ResolutionHeight = height;
    m_FrameSeed = 0;
    return true;
}

bool CScene::LoadFromFile(const char* path)
{
    if (!m_Handle || dcrt_scene_load_from_file(m_Handle, path) != DCRT_OK) return false;
    return dcrt_scene_get_resolution(m_Handle, &m_ResolutionWidth, &m_ResolutionHeight) == DCRT_OK;
}

// ---- the constant / buffer / filter helpers -------------------------------------------------
dcrt_frame_params MakeFrameParams(const CScene& scene, const SRenderContext& renderContext)
{
    dcrt_frame_params p;
    std::memset(&p, 0, sizeof(p));
    (void)dcrt_scene_get_frame_params(scene.m_Handle, scene.m_FrameSeed, &p);   // g_FrameSeed = m_FrameSeed (:412)
    if (renderContext.m_CurrentResolutionWidth && renderContext.m_CurrentResolutionHeight) {
        // g_Resolution / g_FilmDimension = the render context's current resolution (:380-402)
        p.resolution[0] = renderContext.m_CurrentResolutionWidth;
        p.resolution[1] = renderContext.m_CurrentResolutionHeight;
    }
    return p;
}

dcrt_flat_scene MakeFlatScene(const CScene& scene)
{
    dcrt_flat_scene flat;
    std::memset(&flat, 0, sizeof(flat));
    (void)dcrt_scene_get_flat(scene.m_Handle, &flat);
    return flat;
}

dcrt_filter_params MakeFilter(const CScene& scene)
{
    dcrt_filter_params f;
    std::memset(&f, 0, sizeof(f));
    (void)dcrt_scene_get_filter(scene.m_Handle, &f);
    return f;
}

// ---- CMI355XPathTracer ---------------------------------------------------------------------
CMI355XPathTracer::CMI355XPathTracer(uint32_t pathPoolSize, uint32_t iterationsPerFrame, int device)
    : m_PathPoolSize(pathPoolSize), m_IterationPerFrame(iterationsPerFrame), m_Device(device)
{
}

CMI355XPathTracer::~CMI355XPathTracer() { Destroy(); }

bool CMI355XPathTracer::Ok(int rc, const char* what)
{
    if (rc == DCRT_OK) return true;
    m_LastStatus = rc;
    std::fprintf(stderr, "CMI355XPathTracer: %s failed (%d): %s\n", what, rc, dcrt_last_error());
    return false;
}

bool CMI355XPathTracer::Create()
{
    // the only failure the reference reports (Create() -> false aborts Init, LaunchRendererLoop.cpp:61-64)
    if (dcrt_abi_version() != DCRT_ABI_VERSION) {
        std::fprintf(stderr, "CMI355XPathTracer: libdcrt.so ABI %d, header %d\n", dcrt_abi_version(), DCRT_ABI_VERSION);
        return false;
    }
    dcrt_tracer_config cfg;
    std::memset(&cfg, 0, sizeof(cfg));
    cfg.path_pool_size = m_PathPoolSize;
    cfg.iterations_per_render = m_IterationPerFrame;
    cfg.device = m_Device;
    return Ok(dcrt_tracer_create(&cfg, &m_Tracer), "Create");
}

void CMI355XPathTracer::Destroy()
{
    if (m_Tracer) dcrt_tracer_destroy(m_Tracer);
    m_Tracer = nullptr;
    m_HasScene = false;
}

void CMI355XPathTracer::OnSceneLoaded(CScene* scene)
{
    if (!m_Tracer || !scene) return;
    const dcrt_flat_scene flat = MakeFlatScene(*scene);
    m_HasScene = Ok(dcrt_tracer_upload_scene(m_Tracer, &flat), "OnSceneLoaded");
    if (!m_HasScene) return;
    // the film and sample textures at the scene's resolution (Scene.cpp:851-885)
    const dcrt_frame_params p = MakeFrameParams(*scene, SRenderContext{});
    (void)Ok(dcrt_tracer_set_frame_params(m_Tracer, &p), "SetFrameParams");
    ResetImage();
}

void CMI355XPathTracer::Render(CScene* scene, const SRenderContext& renderContext)
{
    if (!m_Tracer || !m_HasScene || !scene) return;
    const dcrt_frame_params p = MakeFrameParams(*scene, renderContext);
    if (!Ok(dcrt_tracer_set_frame_params(m_Tracer, &p), "SetFrameParams")) return;
    // SET_IDLE on a new image, then m_IterationPerFrame x RenderOneIteration (:441-473)
    (void)Ok(dcrt_tracer_render(m_Tracer, m_IterationPerFrame), "Render");
}

void CMI355XPathTracer::ResetImage()
{
    if (m_Tracer) (void)Ok(dcrt_tracer_reset_image(m_Tracer), "ResetImage");
}

bool CMI355XPathTracer::IsImageComplete()
{
    int complete = 0;
    return m_Tracer && Ok(dcrt_tracer_is_image_complete(m_Tracer, &complete), "IsImageComplete") && complete != 0;
}

bool CMI355XPathTracer::AcquireFilmClearTrigger()
{
    int trigger = 0;
    return m_Tracer && Ok(dcrt_tracer_acquire_film_clear_trigger(m_Tracer, &trigger), "AcquireFilmClearTrigger") && trigger != 0;
}

bool CMI355XPathTracer::ClearFilm() { return m_Tracer && Ok(dcrt_tracer_clear_film(m_Tracer), "ClearFilm"); }

bool CMI355XPathTracer::ExecuteSampleConvolution(const dcrt_filter_params& filter)
{
    return m_Tracer && Ok(dcrt_tracer_accumulate_film(m_Tracer, &filter), "SampleConvolution");
}

bool CMI355XPathTracer::GetSampleTextures(void** devicePosition, void** deviceValue)
{
    return m_Tracer && Ok(dcrt_tracer_sample_device_ptrs(m_Tracer, devicePosition, deviceValue), "SampleTextures");
}
