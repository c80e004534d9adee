// mi355x_path_tracer.h -- the reference's path-tracer plugin slot, filled by the MI355X tracer.
//
// This is the drop-in as the reference's application sees it: the `CPathTracer` interface of
// Source/PathTracer.h:6-26 (eight virtuals, restated here because the reference header cannot be
// compiled on Linux), `SRenderContext` (Source/RenderContext.h:1-8), the members of `CScene` the
// frame loop and the plugin read (Source/Scene.h: m_ResolutionWidth/Height, m_FrameSeed,
// m_IsFilmDirty, m_IsLastFrameFilmDirty, m_PathTracer[]), and `CMI355XPathTracer`, a CPathTracer
// that forwards to libdcrt.so through the C ABI of include/dcrt.h alone.
//
// On the reference side a maintainer drops CMI355XPathTracer next to CWavefrontPathTracer and
// deletes the restated declarations below in favour of the real PathTracer.h / Scene.h
// (INTEGRATION.md). The scene content itself lives in the kept host API (dcrt_scene: CScene's
// loaders, BVHAccel and flattening, Scene.cpp:103-624), which `CScene::m_Handle` owns.
#pragma once

#include <cstdint>

#include "dcrt.h"

// Source/RenderContext.h:1-8
struct SRenderContext {
    uint32_t m_CurrentResolutionWidth = 0;
    uint32_t m_CurrentResolutionHeight = 0;
    float m_CurrentResolutionRatio = 1.0f;
    bool m_IsSmallResolutionEnabled = false;
};

class CScene;

// Source/PathTracer.h:6-26 -- the plugin slot (CScene::m_PathTracer[], Scene.h:209)
class CPathTracer {
public:
    virtual ~CPathTracer() {}
    virtual bool Create() = 0;
    virtual void Destroy() {}
    virtual void OnSceneLoaded(CScene* scene) { (void)scene; }
    virtual void Render(CScene* scene, const SRenderContext& renderContext) { (void)scene; (void)renderContext; }
    virtual void ResetImage() {}
    virtual bool IsImageComplete() = 0;
    virtual void OnImGUI(CScene* scene) { (void)scene; }
    virtual bool AcquireFilmClearTrigger() = 0;
};

// The CScene members the frame loop (LaunchRendererLoop.cpp:201-264) and the plugin
// (WavefrontPathTracer.cpp:363-428) read; the content is the kept host scene (dcrt_scene).
class CScene {
public:
    CScene();
    ~CScene();
    CScene(const CScene&) = delete;
    CScene& operator=(const CScene&) = delete;

    // CScene::Reset (Scene.cpp:626-660) + LoadFromFile (Scene.cpp:103-624)
    bool Reset(uint32_t width, uint32_t height);
    bool LoadFromFile(const char* path);

    dcrt_scene* m_Handle = nullptr;
    uint32_t m_ResolutionWidth = 0;
    uint32_t m_ResolutionHeight = 0;
    uint32_t m_FrameSeed = 0;             // Scene.h:138, advanced by the frame loop's seed policy
    bool m_IsFilmDirty = false;
    bool m_IsLastFrameFilmDirty = false;
    // UpdateLight/Material/InstanceFlagsGPUData (Scene.cpp:672-807): the frame loop re-uploads
    // the scene buffers when the host scene was edited
    bool m_IsSceneGPUBufferDirty = false;
    CPathTracer* m_PathTracer[2] = {nullptr, nullptr};
};

// The constants CWavefrontPathTracer::Render uploads (WavefrontPathTracer.cpp:372-428): the
// scene's camera / lens / lights with g_FrameSeed = scene->m_FrameSeed (:412) and the dispatch
// resolution of the render context (:380-402).
dcrt_frame_params MakeFrameParams(const CScene& scene, const SRenderContext& renderContext);
// The buffers Scene.cpp:273-608 uploads (SURVEY Appendix B layouts); valid until the scene changes.
dcrt_flat_scene MakeFlatScene(const CScene& scene);
// The scene's reconstruction filter (Scene.h:131-136), as ExecuteSampleConvolution reads it
// (SampleConvolution.cpp:100-130).
dcrt_filter_params MakeFilter(const CScene& scene);

// CPathTracer backed by the MI355X wavefront tracer (libdcrt.so).
class CMI355XPathTracer : public CPathTracer {
public:
    explicit CMI355XPathTracer(uint32_t pathPoolSize = 1u << 21, uint32_t iterationsPerFrame = 16, int device = 0);
    ~CMI355XPathTracer() override;

    bool Create() override;                                   // CWavefrontPathTracer::Create (:70-300)
    void Destroy() override;
    void OnSceneLoaded(CScene* scene) override;               // scene upload (Scene.cpp:273-608) + :345
    void Render(CScene* scene, const SRenderContext& renderContext) override;   // :363-501
    void ResetImage() override;                               // :503-506
    bool IsImageComplete() override;                          // :508-523 (exact here, not 2 frames late)
    bool AcquireFilmClearTrigger() override;

    // What the application's L1 passes need from the tracer: the film (the tracer owns it on
    // the device) and the current image's sample textures (SampleConvolution's inputs).
    bool ClearFilm();                                         // ClearFilmTexture (LaunchRendererLoop.cpp:192-199)
    bool ExecuteSampleConvolution(const dcrt_filter_params& filter);   // SampleConvolution.cpp:89-170
    bool GetSampleTextures(void** devicePosition, void** deviceValue); // m_SamplePosition/ValueTexture
    dcrt_tracer* GetTracer() const { return m_Tracer; }
    int LastStatus() const { return m_LastStatus; }

private:
    bool Ok(int rc, const char* what);

    dcrt_tracer* m_Tracer = nullptr;
    uint32_t m_PathPoolSize;
    uint32_t m_IterationPerFrame;                             // WavefrontPathTracer.h:84 (reference default 2)
    int m_Device;
    bool m_HasScene = false;
    int m_LastStatus = DCRT_OK;
};
