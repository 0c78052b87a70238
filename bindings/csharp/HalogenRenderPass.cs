// HalogenRenderPass.cs — drop-in replacement for Assets/Scripts/Render Features/HalogenRenderPass.cs ("RP") whose
// GPU work runs in libhalogen_hip (MI355X, gfx950) through HalogenNative (P/Invoke of include/halogen_abi.h).
//
// Kept from the reference, with the same meaning: the class name, base class and public surface (constructor from
// HalogenSettings, OnCameraSetup, Execute, Dispose, getFrameCount; tests/test_csharp_render_pass.py compares it with
// the reference's), the settings clamping (RP:169-231), the camera / resolution / Accumulate bookkeeping that resets
// FrameCount (RP:253-291), the scene gathering from RayTracingManager with material de-duplication and buffer offsets
// (RP:448-537), the uniform values (RP:359-401) and the MaxAccumulatedFrames / UnlimitedSampling rule (RP:307-318).
// Replaced: ComputeShader / ComputeBuffer / RTHandle work and the accumulation blit.  The library traces and blends
// (acc*(1-w) + new*w, w = 1/FrameCount, fused), so the pass keeps one display texture per camera size and uploads
// the accumulated image into it.  The record structs live in HalogenStructs.cs.
//
// Multi-GPU (not in the reference): with HALOGEN_GPUS=n (n > 1) the pass opens one context per device 0..n-1, deals
// the image's 8x8 tiles to them (hg_set_tiling) and gathers the accumulated tiles to device 0 once per displayed
// frame over RCCL (hg_comm_init_all / hg_comm_gather); the image is identical to a one-GPU render.
//
// Display (RP:343-347): each frame's display readback is enqueued on the GPU (hg_readback_begin_format, or
// hg_comm_readback_begin after the gather) and the image of HALOGEN_DISPLAY_LATENCY frames ago is shown: 0, the
// default, is the reference's (the frame just traced, RP:343-345); k > 0 opts into showing k frames behind while the
// next frames trace.  After a ClearAccumulation the readbacks in flight are ended unseen and the next frame is shown at
// once, so an image from before a camera move is never shown.  The image comes in the format of the reference's camera
// target, R11G11B10 float (URP-HighFidelity.asset:26-27, 4 B per pixel; HALOGEN_DISPLAY_FORMAT = r11g11b10f | rgba16f |
// rgba32f; any other value is an error), packed on the GPU; the fp32 accumulation target itself is never changed.
//
// No C# toolchain exists in the build image: this file is checked textually (public surface, the ABI calls it makes
// exist in HalogenNative.cs and the header), not compiled.
using System;
using System.Collections.Generic;
using System.Linq;
using System.Runtime.InteropServices;
using Unity.Mathematics;
using UnityEngine;
using UnityEngine.Experimental.Rendering;
using UnityEngine.Rendering;
using UnityEngine.Rendering.Universal;

public class HalogenRenderPass : ScriptableRenderPass
{
    // ---------------------------------------------------------------- settings (clamped once, RP:169-231)
    struct PassSettings
    {
        public int spp, bounces, diffuse, glossy, transmission, maxFrames, mipLevel, debugMode, triRange, boxRange;
        public float filterRadius, focalDistance, nearPlane, farPlane, aperture;
        public bool accumulate, unlimited, useCubemap;
        public Cubemap cubemap;
    }

    static PassSettings Clamp(HalogenSettings s)
    {
        var p = new PassSettings
        {
            spp = Mathf.Max(1, s.SamplesPerPixel),
            bounces = Mathf.Max(0, s.MaxBounces),
            diffuse = Mathf.Max(0, s.DiffuseBounces),
            glossy = Mathf.Max(0, s.GlossyBounces),
            transmission = Mathf.Max(0, s.TransmissionBounces),
            filterRadius = Mathf.Max(0, s.FilterRadius),
            focalDistance = Mathf.Max(Mathf.Epsilon, s.FocalPlaneDistance),
            nearPlane = Mathf.Max(Mathf.Epsilon, s.NearPlaneDistance),
            aperture = Mathf.Clamp(s.ApertureAngle, 0, 89.9f),
            mipLevel = math.clamp(s.EnvironmentMipLevel, 0, 2),
            accumulate = s.Accumulate,
            maxFrames = math.max(s.MaxAccumulatedFrames, 1),
            unlimited = s.UnlimitedSampling,
            useCubemap = s.useHDRISky && s.environmentCubemap != null,
            cubemap = s.environmentCubemap,
            triRange = Mathf.Max(s.TriangleDebugDisplayRange, 1),
            boxRange = Mathf.Max(s.BoxDebugDisplayRange, 1),
        };
        p.farPlane = Mathf.Max(p.nearPlane + Mathf.Epsilon, s.FarPlaneDistance);
        p.debugMode = DebugModeIndex(s.DebugMode);
        if (p.debugMode != 0 && s.FirstInteractionOnly) p.bounces = 0;
        return p;
    }

    static int DebugModeIndex(HalogenDebugMode mode)
    {
        if (mode == HalogenDebugMode.Albedo) return 1;
        if (mode == HalogenDebugMode.Normal) return 2;
        if (mode == HalogenDebugMode.RayTriangleTests) return 3;
        if (mode == HalogenDebugMode.RayBoxTests) return 4;
        if (mode == HalogenDebugMode.Combined) return 5;
        return 0;
    }

    readonly PassSettings cfg;

    // ---------------------------------------------------------------- native state
    readonly IntPtr[] contexts;      // one hg_ctx per GPU
    IntPtr comm = IntPtr.Zero;       // hg_comm over the contexts when there are several
    bool cubemapUploaded;
    bool disposed;

    // ---------------------------------------------------------------- host bookkeeping (RP:92-152)
    int FrameCount = 1;
    bool AccumulationBufferDirty = true;
    bool ObjectBuffersDirty = true;
    Vector3 PriorCameraPosition;
    Quaternion PriorCameraRotation;
    Vector2Int PriorResolution;
    int sceneSpheres, sceneMeshes;

    RTHandle rtDisplay;              // what the camera sees: the accumulated (or single) frame
    Texture2D uploadTexture;         // staging for the read-back image, in the display format
    bool haveImage;
    readonly int displayFormat;      // HG_DISPLAY_* (HALOGEN_DISPLAY_FORMAT)
    readonly int displayLatency;     // frames the shown image lags the traced one (HALOGEN_DISPLAY_LATENCY)
    int displayPending;              // display readbacks enqueued and not yet shown
    bool displayResync;              // the first frame after a clear is shown at once
    readonly ProfilingSampler sampler = new ProfilingSampler("Halogen (MI355X)");

    // scene lists, rebuilt by UpdateObjectBuffers
    readonly List<HalogenSphere> spheres = new List<HalogenSphere>();
    readonly List<HalogenMeshData> meshes = new List<HalogenMeshData>();
    readonly List<PackedHalogenMaterial> packedMaterials = new List<PackedHalogenMaterial>();
    readonly List<HalogenTriangle> triangles = new List<HalogenTriangle>();
    readonly List<BVHEntry> blas = new List<BVHEntry>();
    readonly List<HalogenMaterial> seenMaterials = new List<HalogenMaterial>();
    // the geometry generation of hg_upload_scene_gen: bumped whenever the mesh registry's members (manager ID, triangle
    // count, BVH size, in order) differ from the last upload's; equal, it vouches for the 78 MB of triangles and BVH
    // entries the reference re-uploads on every camera move (RP:262-268, 296-299), which the library then skips comparing
    readonly List<long> geometrySignature = new List<long>();
    ulong geometryGeneration;

    public HalogenRenderPass(ref HalogenSettings _settings)
    {
        UnityEditor.AssemblyReloadEvents.beforeAssemblyReload += () => { Dispose(); };
        cfg = Clamp(_settings);

        int gpus = 1;
        int.TryParse(Environment.GetEnvironmentVariable("HALOGEN_GPUS") ?? "1", out gpus);
        gpus = Math.Max(1, gpus);
        contexts = new IntPtr[gpus];
        for (int d = 0; d < gpus; d++)
        {
            int rc = HalogenNative.hg_create(d, out contexts[d]);
            if (rc != HalogenNative.HG_OK) throw new Exception($"hg_create({d}) failed ({rc}): no usable MI355X device");
            // the pass never reads the work counters (the reference has none); off, the render server may trace the
            // next frames of an unchanged camera ahead of the calls (HG_OPT_SERVER_AHEAD)
            Check(HalogenNative.hg_set_option(contexts[d], HalogenNative.HG_OPT_COUNTERS, 0), "hg_set_option(HG_OPT_COUNTERS)");
        }

        string fmt = (Environment.GetEnvironmentVariable("HALOGEN_DISPLAY_FORMAT") ?? "r11g11b10f").ToLowerInvariant();
        if (fmt == "rgba32f") displayFormat = HalogenNative.HG_DISPLAY_RGBA32F;
        else if (fmt == "rgba16f") displayFormat = HalogenNative.HG_DISPLAY_RGBA16F;
        else if (fmt == "r11g11b10f") displayFormat = HalogenNative.HG_DISPLAY_R11G11B10F;
        else throw new ArgumentException($"HALOGEN_DISPLAY_FORMAT '{fmt}': expected r11g11b10f, rgba16f or rgba32f");
        string lat = Environment.GetEnvironmentVariable("HALOGEN_DISPLAY_LATENCY") ?? "0";
        if (!int.TryParse(lat, out int latency) || latency < 0 || latency >= HalogenNative.HG_READBACK_MAX)
            throw new ArgumentException($"HALOGEN_DISPLAY_LATENCY '{lat}': expected 0..{HalogenNative.HG_READBACK_MAX - 1}");
        displayLatency = latency;
        // the display ring lives on the context that displays (device 0; the gather's root)
        Check(HalogenNative.hg_set_option(contexts[0], HalogenNative.HG_OPT_READBACK_DEPTH, displayLatency + 1),
              "hg_set_option(HG_OPT_READBACK_DEPTH)");
    }

    GraphicsFormat DisplayGraphicsFormat()
    {
        if (displayFormat == HalogenNative.HG_DISPLAY_RGBA32F) return GraphicsFormat.R32G32B32A32_SFloat;
        if (displayFormat == HalogenNative.HG_DISPLAY_RGBA16F) return GraphicsFormat.R16G16B16A16_SFloat;
        return GraphicsFormat.B10G11R11_UFloatPack32;  // DXGI_FORMAT_R11G11B10_FLOAT: R in bits 0-10
    }

    ~HalogenRenderPass() { Dispose(); }

    void Check(int rc, string what) { HalogenNative.Check(contexts[0], rc, what); }

    // ---------------------------------------------------------------- camera target (RP:237-260)
    public override void OnCameraSetup(CommandBuffer cmd, ref RenderingData renderingData)
    {
        var desc = renderingData.cameraData.cameraTargetDescriptor;
        desc.enableRandomWrite = false;
        desc.bindMS = false;
        desc.depthBufferBits = 0;
        desc.graphicsFormat = DisplayGraphicsFormat();
        RenderingUtils.ReAllocateIfNeeded(ref rtDisplay, desc, name: "_HalogenDisplay");

        var size = new Vector2Int(desc.width, desc.height);
        if (size == PriorResolution) return;
        PriorResolution = size;
        for (int r = 0; r < contexts.Length; r++)
        {
            Check(HalogenNative.hg_resize(contexts[r], size.x, size.y), "hg_resize");
            Check(HalogenNative.hg_set_tiling(contexts[r], r, contexts.Length), "hg_set_tiling");
        }
        if (contexts.Length > 1 && comm == IntPtr.Zero)
        {
            int rc = HalogenNative.hg_comm_init_all(contexts, contexts.Length, out comm);
            Check(rc, "hg_comm_init_all");
        }
        if (uploadTexture != null) UnityEngine.Object.DestroyImmediate(uploadTexture);
        uploadTexture = new Texture2D(size.x, size.y, DisplayGraphicsFormat(), TextureCreationFlags.None);
        haveImage = false;
        displayPending = 0;  // hg_resize / hg_set_tiling dropped the display readbacks in flight
        ClearAccumulation();
    }

    void ClearAccumulation()
    {
        FrameCount = 1;
        AccumulationBufferDirty = true;
        ObjectBuffersDirty = true;
        DropDisplay();
    }

    // The display readbacks in flight show images from before a clear: end them unseen, and show the next frame at once
    void DropDisplay()
    {
        for (; displayPending > 0; displayPending--)
        {
            IntPtr image;
            UIntPtr nBytes;
            int format;
            int rc = comm != IntPtr.Zero ? HalogenNative.hg_comm_readback_end(comm, out image, out nBytes, out format)
                                         : HalogenNative.hg_readback_end_data(contexts[0], out image, out nBytes, out format);
            if (rc != HalogenNative.HG_OK) throw new Exception($"display readback failed ({rc})");
        }
        displayResync = displayLatency > 0;
    }

    // ---------------------------------------------------------------- one frame (RP:270-357)
    public override void Execute(ScriptableRenderContext context, ref RenderingData renderingData)
    {
        Camera camera = renderingData.cameraData.camera;
        Transform view = camera.transform;

        // any camera move restarts accumulation; so does a frame after the first with Accumulate off
        bool moved = !PriorCameraPosition.Equals(view.position) || !PriorCameraRotation.Equals(view.rotation);
        if (moved || (FrameCount > 1 && !cfg.accumulate)) ClearAccumulation();
        PriorCameraPosition = view.position;
        PriorCameraRotation = view.rotation;

        if (ObjectBuffersDirty)
        {
            UpdateObjectBuffers();
            ObjectBuffersDirty = false;
        }

        CommandBuffer cmd = CommandBufferPool.Get("HalogenPass");
        using (new ProfilingScope(cmd, sampler))
        {
            bool finished = !cfg.unlimited && FrameCount > cfg.maxFrames;
            if (!finished)
            {
                TraceOneFrame(camera);
                if (cfg.accumulate) FrameCount++;
            }
            if (haveImage)
                Blitter.BlitCameraTexture(cmd, rtDisplay, renderingData.cameraData.renderer.cameraColorTargetHandle);
        }
        context.ExecuteCommandBuffer(cmd);
        CommandBufferPool.Release(cmd);
    }

    // The uniform block of DispatchHalogenTrace (RP:359-401) and one hg_render per context; the library fuses the
    // accumulation blend (AccumulationShader.shader:33) into the trace.
    void TraceOneFrame(Camera camera)
    {
        float halfHeight = Mathf.Tan(Mathf.Deg2Rad * camera.fieldOfView * 0.5f) * cfg.nearPlane;
        var p = new HalogenNative.HgParams
        {
            camLocalToWorld = camera.transform.localToWorldMatrix,
            screenParameters = new Vector4(camera.pixelWidth, camera.pixelHeight, 0, 0),
            viewParameters = new Vector4(camera.aspect * halfHeight, halfHeight, cfg.nearPlane, cfg.farPlane),
            cameraParameters = camera.transform.position,
            frameCount = cfg.accumulate ? FrameCount : 1,
            samplesPerPixel = (uint)cfg.spp,
            maxBounces = (uint)cfg.bounces,
            maxDiffuseBounces = (uint)cfg.diffuse,
            maxGlossyBounces = (uint)cfg.glossy,
            maxTransmissionBounces = (uint)cfg.transmission,
            halogenDebugMode = (uint)cfg.debugMode,
            triangleDebugDisplayRange = (uint)cfg.triRange,
            boxDebugDisplayRange = (uint)cfg.boxRange,
            defaultHDRIMipLevel = cfg.mipLevel,
            focalPlaneDistance = cfg.focalDistance,
            focalConeAngle = cfg.aperture,
            filterRadius = cfg.filterRadius,
            useEnvironmentCubemap = cfg.useCubemap ? 1 : 0,
            bufferCounts = new Vector4(sceneSpheres, sceneMeshes, 0, 0),
        };
        foreach (IntPtr ctx in contexts)
        {
            Check(HalogenNative.hg_set_params(ctx, ref p), "hg_set_params");
            if (AccumulationBufferDirty) Check(HalogenNative.hg_clear_accumulation(ctx), "hg_clear_accumulation");
            Check(HalogenNative.hg_render(ctx, 1, cfg.accumulate ? 1 : 0), "hg_render");  // asynchronous per GPU
        }
        AccumulationBufferDirty = false;

        // the display image (RP:343-347), pipelined: enqueue this frame's readback on the GPU and show the one of
        // `displayLatency` frames ago; with several GPUs the gather to device 0 comes first (bounded waits throughout)
        int rc;
        if (comm != IntPtr.Zero)
        {
            rc = HalogenNative.hg_comm_gather(comm, 0);
            if (rc == HalogenNative.HG_OK) rc = HalogenNative.hg_comm_readback_begin(comm, displayFormat);
            if (rc != HalogenNative.HG_OK)
                throw new Exception($"multi-GPU gather failed ({rc}): {Marshal.PtrToStringAnsi(HalogenNative.hg_comm_last_error(comm))}");
        }
        else
        {
            Check(HalogenNative.hg_readback_begin_format(contexts[0], displayFormat), "hg_readback_begin_format");
        }
        displayPending++;
        if (displayResync)  // the first frame after a clear: its own image at once (the older ones were dropped)
            displayResync = false;
        else if (displayPending <= displayLatency)
            return;  // the pipeline fills: keep showing the previous image
        IntPtr image;
        UIntPtr nBytes;
        int format;
        if (comm != IntPtr.Zero)
        {
            rc = HalogenNative.hg_comm_readback_end(comm, out image, out nBytes, out format);
            if (rc != HalogenNative.HG_OK)
                throw new Exception($"multi-GPU display failed ({rc}): {Marshal.PtrToStringAnsi(HalogenNative.hg_comm_last_error(comm))}");
        }
        else
        {
            Check(HalogenNative.hg_readback_end_data(contexts[0], out image, out nBytes, out format), "hg_readback_end_data");
        }
        displayPending--;
        uploadTexture.LoadRawTextureData(image, checked((int)nBytes.ToUInt64()));
        uploadTexture.Apply(false);
        Graphics.Blit(uploadTexture, rtDisplay);
        haveImage = true;
    }

    // ---------------------------------------------------------------- scene buffers (RP:448-509)
    void UpdateObjectBuffers()
    {
        spheres.Clear();
        meshes.Clear();
        packedMaterials.Clear();
        triangles.Clear();
        blas.Clear();
        seenMaterials.Clear();

        foreach (RayTracingSphere s in RayTracingManager.GetSphereList().Values)
        {
            Vector3 c = s.transform.position;
            float r = s.GetRadius();
            spheres.Add(new HalogenSphere
            {
                center = c, radius = r, materialIndex = MaterialSlot(s.material),
                boundingCornerA = c - Vector3.one * r, boundingCornerB = c + Vector3.one * r,
            });
        }
        var signature = new List<long>();
        foreach (RayTracingMesh m in RayTracingManager.GetMeshList().Values)
        {
            uint mat = MaterialSlot(m.material);
            uint triOffset = (uint)triangles.Count, nodeOffset = (uint)blas.Count;
            triangles.AddRange(m.GetPackedTriangles());
            meshes.Add(m.GetRefreshedMeshData(mat, triOffset, nodeOffset));
            blas.AddRange(m.GetBVH());
            signature.Add(m.GetID());  // new on every OnEnable, when the mesh re-reads its triangles (RayTracingManager.cs:74-79)
            signature.Add(triangles.Count - triOffset);
            signature.Add(blas.Count - nodeOffset);
        }
        if (geometryGeneration == 0 || !signature.SequenceEqual(geometrySignature))
        {
            geometryGeneration++;
            geometrySignature.Clear();
            geometrySignature.AddRange(signature);
        }
        sceneSpheres = spheres.Count;
        sceneMeshes = meshes.Count;

        // the library copies the arrays during the call (SetBufferData semantics); every GPU holds the whole scene
        HalogenSphere[] sph = spheres.ToArray();
        HalogenMeshData[] msh = meshes.ToArray();
        PackedHalogenMaterial[] mats = packedMaterials.ToArray();
        HalogenTriangle[] tris = triangles.ToArray();
        BVHEntry[] nodes = blas.ToArray();
        foreach (IntPtr ctx in contexts)
        {
            Check(HalogenNative.hg_upload_scene_gen(ctx, geometryGeneration, sph, sph.Length, msh, msh.Length, mats,
                                                    mats.Length, tris, tris.Length, nodes, nodes.Length),
                  "hg_upload_scene_gen");
            if (cfg.useCubemap && !cubemapUploaded) UploadCubemap(ctx);
        }
        cubemapUploaded = cfg.useCubemap;
    }

    // Index of `material` in the packed list, packing it on first use (PackMaterialToList, RP:524-537: equality by
    // value, so identical materials share one slot).
    uint MaterialSlot(HalogenMaterial material)
    {
        int found = seenMaterials.IndexOf(material);
        if (found >= 0) return (uint)found;
        int id = packedMaterials.Count;
        seenMaterials.Add(material);
        packedMaterials.Add(Pack(material, id));
        return (uint)id;
    }

    // PackHalogenMaterial (RP:425-446): albedo / specular as the raw colour (linear project), emission (rgb,
    // intensity), absorption = (1 / subsurface colour) * max(absorption, 0).
    static PackedHalogenMaterial Pack(HalogenMaterial m, int id)
    {
        Vector4 sub = m.subsurfaceColor;
        float k = Mathf.Max(m.absorption, 0);
        return new PackedHalogenMaterial
        {
            materialID = (uint)id,
            albedo = m.color,
            specularAlbedo = m.specularColor,
            metallic = m.metallic,
            roughness = m.roughness,
            emissive = new Vector4(m.emissionColor.r, m.emissionColor.g, m.emissionColor.b, m.emissionIntensity),
            rayMedium = new PackedRayMedium
            {
                indexOfRefraction = m.indexOfRefraction,
                absorption = new Vector3(1 / sub.x, 1 / sub.y, 1 / sub.z) * k,
                priority = m.dielectricPriority,
                materialID = (uint)id,
            },
        };
    }

    // hg_upload_cubemap takes RGBA32F texels [mip][face][y][x] with row 0 at the top of each face (D3D face
    // orientation, faces +X,-X,+Y,-Y,+Z,-Z); Unity's GetPixels rows start at the bottom, so rows are flipped.
    void UploadCubemap(IntPtr ctx)
    {
        Cubemap cube = cfg.cubemap;
        int size = cube.width, mips = cube.mipmapCount;
        var texels = new List<float>();
        for (int mip = 0; mip < mips; mip++)
        {
            int s = Math.Max(1, size >> mip);
            for (int face = 0; face < 6; face++)
            {
                Color[] px = cube.GetPixels((CubemapFace)face, mip);
                for (int y = s - 1; y >= 0; y--)
                    for (int x = 0; x < s; x++)
                    {
                        Color c = px[y * s + x];
                        texels.Add(c.r); texels.Add(c.g); texels.Add(c.b); texels.Add(c.a);
                    }
            }
        }
        float[] data = texels.ToArray();
        Check(HalogenNative.hg_upload_cubemap(ctx, size, mips, data, (UIntPtr)data.Length), "hg_upload_cubemap");
    }

    // ---------------------------------------------------------------- release (RP:410-423)
    public void Dispose()
    {
        if (disposed) return;
        disposed = true;
        if (comm != IntPtr.Zero) HalogenNative.hg_comm_destroy(comm);
        comm = IntPtr.Zero;
        foreach (IntPtr ctx in contexts)
            if (ctx != IntPtr.Zero) HalogenNative.hg_destroy(ctx);
        rtDisplay?.Release();
        if (uploadTexture != null) UnityEngine.Object.DestroyImmediate(uploadTexture);
    }

    public int getFrameCount()
    {
        return FrameCount;
    }

    // Checkpoint resume (not in the reference, whose resumable state is the accumulation target and FrameCount,
    // RP:152,185,347): after OnCameraSetup at the image's size, Restore(image, frameCount, camera) continues the
    // progressive render bit-identically (hg_set_accumulation; with several GPUs each context takes its own tiles).
    // internal, so the public surface stays the reference's.
    internal void Restore(float[] image, int frameCount, Transform cameraTransform)
    {
        foreach (IntPtr ctx in contexts)
            Check(HalogenNative.hg_set_accumulation(ctx, image, (UIntPtr)image.Length, frameCount), "hg_set_accumulation");
        FrameCount = frameCount;
        AccumulationBufferDirty = false;
        PriorCameraPosition = cameraTransform.position;  // the restored frames' camera: no restart on the next Execute
        PriorCameraRotation = cameraTransform.rotation;
    }
}
