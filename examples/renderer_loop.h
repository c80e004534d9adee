// renderer_loop.h -- the reference's frame loop around the path-tracer plugin, restated for a
// headless host: CDirectComputeRayTracing::LoadScene (LaunchRendererLoop.cpp:159-190),
// HandleFilmResolutionChange's small resolution (:395-410), DispatchRayTracing (:201-270) and the
// film half of RenderOneFrame (:273-298). Window, ImGui, luminance and post-processing passes
// stay out; the film is convolved exactly when the reference convolves it.
#pragma once

#include <algorithm>
#include <cmath>
#include <cstdint>

#include "mi355x_path_tracer.h"

class CRendererLoop {
public:
    // DirectComputeRayTracing.h:111-112
    enum class EFrameSeedType { FrameIndex = 0, SampleCount = 1, Fixed = 2 };

    CRendererLoop(CScene* scene, CMI355XPathTracer* pathTracer) : m_Scene(scene), m_PathTracer(pathTracer)
    {
        m_Scene->m_PathTracer[0] = pathTracer;
    }

    // LaunchRendererLoop.cpp:159-190: the film is dirty from here on, so the next frame is the
    // small-resolution preview
    bool LoadScene(const char* path, uint32_t width, uint32_t height)
    {
        m_Scene->m_IsFilmDirty = true;
        if (!m_Scene->Reset(width, height) || !m_Scene->LoadFromFile(path)) return false;
        return AfterSceneEdited();
    }
    // the tail of LoadScene after scene content changed (OnSceneLoaded, :175-183)
    bool AfterSceneEdited()
    {
        m_Scene->m_IsFilmDirty = true;
        m_PathTracer->OnSceneLoaded(m_Scene);
        HandleFilmResolutionChange();
        return m_PathTracer->LastStatus() == DCRT_OK;
    }
    // :395-410
    void HandleFilmResolutionChange()
    {
        m_SmallResolutionWidth = std::max(1u, (uint32_t)std::roundf(m_Scene->m_ResolutionWidth * 0.25f));
        m_SmallResolutionHeight = std::max(1u, (uint32_t)std::roundf(m_Scene->m_ResolutionHeight * 0.25f));
    }

    // DispatchRayTracing (:201-270)
    void DispatchRayTracing(SRenderContext* renderContext)
    {
        CScene* scene = m_Scene;
        CPathTracer* pt = scene->m_PathTracer[m_ActivePathTracerIndex];
        scene->m_IsFilmDirty = scene->m_IsFilmDirty || scene->m_IsSceneGPUBufferDirty || pt->AcquireFilmClearTrigger();

        const bool isResolutionChanged = scene->m_IsFilmDirty != scene->m_IsLastFrameFilmDirty;
        renderContext->m_IsSmallResolutionEnabled = scene->m_IsFilmDirty;
        scene->m_IsLastFrameFilmDirty = scene->m_IsFilmDirty;
        renderContext->m_CurrentResolutionWidth =
            renderContext->m_IsSmallResolutionEnabled ? m_SmallResolutionWidth : scene->m_ResolutionWidth;
        renderContext->m_CurrentResolutionRatio = (float)renderContext->m_CurrentResolutionWidth / scene->m_ResolutionWidth;
        renderContext->m_CurrentResolutionHeight =
            renderContext->m_IsSmallResolutionEnabled ? m_SmallResolutionHeight : scene->m_ResolutionHeight;

        if (scene->m_IsFilmDirty || isResolutionChanged) {
            m_PathTracer->ClearFilm();
            if (m_FrameSeedType == EFrameSeedType::SampleCount) scene->m_FrameSeed = 0;
            m_SPP = 0;
            pt->ResetImage();
        }
        // UpdateLight/Material/InstanceFlagsGPUData (:239-252): the edited host scene re-flattened
        // and uploaded
        if (scene->m_IsSceneGPUBufferDirty) pt->OnSceneLoaded(scene);

        pt->Render(scene, *renderContext);

        if (pt->IsImageComplete()) {
            if (m_FrameSeedType != EFrameSeedType::Fixed) scene->m_FrameSeed++;
            ++m_SPP;
        }
        scene->m_IsSceneGPUBufferDirty = false;
        scene->m_IsFilmDirty = false;
    }

    // RenderOneFrame (:273-298): convolve a completed image, or the preview every frame.
    // Returns false when a tracer call failed.
    bool RenderOneFrame(SRenderContext* renderContext)
    {
        *renderContext = SRenderContext{};
        DispatchRayTracing(renderContext);
        CPathTracer* pt = m_Scene->m_PathTracer[m_ActivePathTracerIndex];
        m_LastFrameCompletedImage = pt->IsImageComplete();
        if (m_LastFrameCompletedImage || renderContext->m_IsSmallResolutionEnabled)
            m_PathTracer->ExecuteSampleConvolution(MakeFilter(*m_Scene));
        ++m_FrameIndex;
        return m_PathTracer->LastStatus() == DCRT_OK;
    }

    CScene* m_Scene;
    CMI355XPathTracer* m_PathTracer;
    uint32_t m_ActivePathTracerIndex = 0;
    EFrameSeedType m_FrameSeedType = EFrameSeedType::SampleCount;   // the reference's default
    uint32_t m_SPP = 0;                                             // images in the film (ImGui.cpp:725)
    uint32_t m_SmallResolutionWidth = 480;
    uint32_t m_SmallResolutionHeight = 270;
    uint64_t m_FrameIndex = 0;
    bool m_LastFrameCompletedImage = false;
};
