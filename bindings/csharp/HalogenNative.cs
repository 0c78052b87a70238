// HalogenNative.cs — P/Invoke binding of libhalogen_hip.so (include/halogen_abi.h) for the reference's C# host.
//
// Used by HalogenRenderPass.cs of this directory, the drop-in for Assets/Scripts/Render Features/
// HalogenRenderPass.cs.  The scene records (HalogenSphere, HalogenMeshData, PackedHalogenMaterial, HalogenTriangle,
// BVHEntry) are declared in HalogenStructs.cs with the header's layout; only the uniform block and the counters are
// new here.  tests/test_csharp_binding.py checks this file against the C header (every export declared, struct
// fields in order with matching types); there is no C# toolchain in the build image, so it is not compiled here.
using System;
using System.Runtime.InteropServices;
using UnityEngine;

public static class HalogenNative
{
    const string Lib = "halogen_hip";

    // hg_params: every uniform of HalgoenCompute.compute:26-68,185 as DispatchHalogenTrace sets it (RP:359-401)
    [StructLayout(LayoutKind.Sequential)]
    public struct HgParams
    {
        public Matrix4x4 camLocalToWorld;     // hg_mat4: Unity column-major m00,m10,...
        public Vector4 screenParameters;      // (pixelWidth, pixelHeight, 0, 0)
        public Vector4 viewParameters;        // (w, h, near, far)
        public Vector4 cameraParameters;      // camera position (dead in the kernel)
        public int frameCount;                // FrameCount of the first traced frame
        public uint samplesPerPixel;
        public uint maxBounces;
        public uint maxDiffuseBounces;
        public uint maxGlossyBounces;
        public uint maxTransmissionBounces;
        public uint halogenDebugMode;
        public uint triangleDebugDisplayRange;
        public uint boxDebugDisplayRange;
        public int defaultHDRIMipLevel;
        public float focalPlaneDistance;
        public float focalConeAngle;
        public float filterRadius;
        public int useEnvironmentCubemap;
        public Vector4 bufferCounts;          // (spheres, meshes, 0, 0)
    }

    [StructLayout(LayoutKind.Sequential)]
    public struct HgCounters
    {
        public ulong paths;
        public ulong rays;
        public ulong tri_tests;
        public ulong aabb_tests;
        public ulong mesh_visits;
        public ulong sphere_tests;
        public ulong hits;
        public double kernel_ms;
        public ulong launches;
        public double trace_ms;
        public ulong trace_launches;
        public ulong node_rounds;
        public ulong tri_rounds;
        public ulong last_kernel;
        public ulong trace_cycles;
        public ulong shade_cycles;
        [MarshalAs(UnmanagedType.ByValArray, SizeConst = 4)] public ulong[] shade_detail;
        public ulong shade_rounds;
        public ulong primary_misses;
        public ulong exec_fallbacks;
        public double trace_busy_ms;
        public ulong order_faults;
        public ulong scene_uploads;
        public ulong scene_uploads_skipped;
        public ulong scene_uploads_partial;
        public ulong scene_uploads_vouched;
        public ulong server_launches;
        public ulong server_frames;
        public ulong server_refused;
        public ulong frames_lost;
        public ulong server_ahead;
    }

    public const int HG_OK = 0;
    public const int HG_KERNEL_MEGA = 0, HG_KERNEL_WAVEFRONT = 1, HG_KERNEL_MEGA_REGEN = 2, HG_KERNEL_MEGA_STREAM = 3,
                     HG_KERNEL_MEGA_POOL = 4, HG_KERNEL_AUTO = 5;
    public const int HG_OPT_KERNEL = 1, HG_OPT_BLOCK = 2, HG_OPT_COUNTERS = 3, HG_OPT_TIMING = 4, HG_OPT_REFILL = 5,
                     HG_OPT_FRAME_SPLIT = 6, HG_OPT_DESCENT_T = 7, HG_OPT_TILE_ORDER = 8, HG_OPT_COALESCE = 9,
                     HG_OPT_READBACK_DEPTH = 10, HG_OPT_READBACK_STREAM = 11, HG_OPT_WAVE_UNITS = 12,
                     HG_OPT_LANE_PICK = 14, HG_OPT_SERVER = 15, HG_OPT_SERVER_IDLE_US = 16, HG_OPT_SERVER_GATE_US = 17,
                     HG_OPT_QUEUE_FILL = 18, HG_OPT_SERVER_AHEAD = 19;
    public const int HG_READBACK_MAX = 16;
    // display formats of hg_readback_begin_format / hg_comm_readback_begin: 16 / 8 / 4 bytes per pixel; R11G11B10F is
    // the URP HDR camera target the reference blits into (GraphicsFormat.B10G11R11_UFloatPack32: R in bits 0-10)
    public const int HG_DISPLAY_RGBA32F = 0, HG_DISPLAY_RGBA16F = 1, HG_DISPLAY_R11G11B10F = 2;
    public const int HG_SELFTEST_RCP = 1, HG_SELFTEST_BUILD = 2, HG_BUILD_CHECK_EXEC = 1, HG_BUILD_NO_REGEN_ITEMS = 2;
    public const int HG_COMM_ID_BYTES = 128, HG_COMM_RCCL = 1, HG_COMM_PEER = 2;

    [DllImport(Lib)] public static extern int hg_abi_version();
    [DllImport(Lib)] public static extern int hg_create(int device, out IntPtr ctx);
    [DllImport(Lib)] public static extern void hg_destroy(IntPtr ctx);
    [DllImport(Lib)] public static extern IntPtr hg_last_error(IntPtr ctx);
    [DllImport(Lib)] public static extern int hg_upload_scene(IntPtr ctx,
        HalogenSphere[] spheres, int nSpheres, HalogenMeshData[] meshes, int nMeshes,
        PackedHalogenMaterial[] materials, int nMaterials, HalogenTriangle[] triangles, int nTriangles,
        BVHEntry[] blas, int nNodes);
    [DllImport(Lib)] public static extern int hg_upload_scene_gen(IntPtr ctx, ulong geometryGeneration,
        HalogenSphere[] spheres, int nSpheres, HalogenMeshData[] meshes, int nMeshes,
        PackedHalogenMaterial[] materials, int nMaterials, HalogenTriangle[] triangles, int nTriangles,
        BVHEntry[] blas, int nNodes);
    [DllImport(Lib)] public static extern int hg_upload_cubemap(IntPtr ctx, int faceSize, int nMips, float[] texels,
        UIntPtr nFloats);
    [DllImport(Lib)] public static extern int hg_set_params(IntPtr ctx, ref HgParams p);
    [DllImport(Lib)] public static extern int hg_resize(IntPtr ctx, int width, int height);
    [DllImport(Lib)] public static extern int hg_set_tiling(IntPtr ctx, int rank, int nRanks);
    [DllImport(Lib)] public static extern int hg_clear_accumulation(IntPtr ctx);
    [DllImport(Lib)] public static extern int hg_render(IntPtr ctx, int nFrames, int accumulate);
    [DllImport(Lib)] public static extern int hg_synchronize(IntPtr ctx);
    [DllImport(Lib)] public static extern int hg_readback(IntPtr ctx, float[] rgba, UIntPtr nFloats);
    [DllImport(Lib)] public static extern int hg_readback_begin(IntPtr ctx);
    [DllImport(Lib)] public static extern int hg_readback_end(IntPtr ctx, out IntPtr rgba, out UIntPtr nFloats);
    [DllImport(Lib)] public static extern int hg_readback_begin_format(IntPtr ctx, int format);
    [DllImport(Lib)] public static extern int hg_readback_end_data(IntPtr ctx, out IntPtr data, out UIntPtr nBytes,
        out int format);
    [DllImport(Lib)] public static extern int hg_pack_display(float[] rgba, UIntPtr nPixels, int format, IntPtr output);
    [DllImport(Lib)] public static extern int hg_set_accumulation(IntPtr ctx, float[] rgba, UIntPtr nFloats, int frameCount);
    [DllImport(Lib)] public static extern int hg_copy_tiles_device(IntPtr ctx, IntPtr dstDevice, UIntPtr nBytes);
    [DllImport(Lib)] public static extern int hg_local_tile_count(IntPtr ctx);
    [DllImport(Lib)] public static extern int hg_get_counters(IntPtr ctx, out HgCounters c);
    [DllImport(Lib)] public static extern int hg_reset_counters(IntPtr ctx);
    [DllImport(Lib)] public static extern int hg_set_option(IntPtr ctx, int option, int value);
    [DllImport(Lib)] public static extern long hg_selftest(IntPtr ctx, int test, out long tested);
    [DllImport(Lib)] public static extern long hg_build_blas(float[] vertices, int nVertices, int[] indices, int nTris,
        float[] rootMin, float[] rootMax, int maxHierarchyDepth, [Out] BVHEntry[] outNodes, long maxNodes);
    [DllImport(Lib)] public static extern long hg_build_blas_mt(float[] vertices, int nVertices, int[] indices,
        int nTris, float[] rootMin, float[] rootMax, int maxHierarchyDepth, [Out] BVHEntry[] outNodes, long maxNodes,
        int nThreads);
    // an SAH hierarchy in the same format: NOT BVHGenerator's tree (a faster render, not the reference's images)
    [DllImport(Lib)] public static extern long hg_build_blas_sah(float[] vertices, int nVertices, int[] indices,
        int nTris, int maxLeaf, int maxDepth, [Out] BVHEntry[] outNodes, long maxNodes);
    [DllImport(Lib)] public static extern void hg_unity_bounds(float[] inMin, float[] inMax, int padIfThin,
        [Out] float[] outMin, [Out] float[] outMax);
    [DllImport(Lib)] public static extern int hg_pack_triangles(float[] vertices, float[] normals, int nVertices,
        int[] indices, int nTris, [Out] HalogenTriangle[] outTriangles);

    // Multi-GPU gather (one context per GPU; the render pass keeps one HalogenRenderPass per device and gathers the
    // tiles to the display device once per displayed image).
    [DllImport(Lib)] public static extern int hg_comm_unique_id([Out] byte[] id);
    [DllImport(Lib)] public static extern int hg_comm_init_rank(IntPtr ctx, int nRanks, byte[] id, int rank,
        out IntPtr comm);
    [DllImport(Lib)] public static extern int hg_comm_init_all(IntPtr[] ctxs, int nRanks, out IntPtr comm);
    [DllImport(Lib)] public static extern int hg_comm_gather(IntPtr comm, int root);
    [DllImport(Lib)] public static extern int hg_comm_synchronize(IntPtr comm);
    [DllImport(Lib)] public static extern int hg_comm_readback(IntPtr comm, float[] rgba, UIntPtr nFloats);
    [DllImport(Lib)] public static extern int hg_comm_readback_begin(IntPtr comm, int format);
    [DllImport(Lib)] public static extern int hg_comm_readback_end(IntPtr comm, out IntPtr data, out UIntPtr nBytes,
        out int format);
    [DllImport(Lib)] public static extern int hg_comm_set_timeout_ms(IntPtr comm, long timeoutMs);
    [DllImport(Lib)] public static extern int hg_comm_transport(IntPtr comm);
    [DllImport(Lib)] public static extern IntPtr hg_comm_last_error(IntPtr comm);
    [DllImport(Lib)] public static extern void hg_comm_destroy(IntPtr comm);
    [DllImport(Lib)] public static extern int hg_comm_assemble_host(float[] slabs, long slabTiles, int width,
        int height, int nRanks, [Out] float[] rgba, UIntPtr nFloats);

    public static void Check(IntPtr ctx, int rc, string what)
    {
        if (rc != HG_OK)
            throw new Exception($"{what} failed ({rc}): {Marshal.PtrToStringAnsi(hg_last_error(ctx))}");
    }
}
