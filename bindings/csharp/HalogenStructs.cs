// HalogenStructs.cs — the scene records the render pass hands to libhalogen_hip, with the byte layout the C-ABI
// declares (include/halogen_abi.h; strides 44 / 164 / 24 / 84 / 72 / 32 B, checked by tests/test_abi.py against the
// header).  The reference declares the same records at the top of HalogenRenderPass.cs (RP:10-76) with default
// (sequential) layout; HalogenRenderPass.cs of this binding no longer holds them, so they live here, with the
// layout made explicit because they now cross a P/Invoke boundary.
using System.Runtime.InteropServices;
using UnityEngine;

[StructLayout(LayoutKind.Sequential)]
public struct HalogenSphere                 // 44 B
{
    public Vector3 center;
    public float radius;
    public uint materialIndex;
    public Vector3 boundingCornerA;         // center - radius (RP:468)
    public Vector3 boundingCornerB;         // center + radius (RP:469)
}

[System.Serializable]
[StructLayout(LayoutKind.Sequential)]
public struct HalogenMeshData               // 164 B
{
    public uint triangleBufferOffset;
    public uint accelerationBufferOffset;
    public Vector3 boundingCornerA;
    public Vector3 boundingCornerB;
    public uint materialIndex;
    public Matrix4x4 worldToLocal;
    public Matrix4x4 localToWorld;
}

[StructLayout(LayoutKind.Sequential)]
public struct PackedRayMedium               // 24 B
{
    public float indexOfRefraction;
    public Vector3 absorption;
    public int priority;
    public uint materialID;
}

[StructLayout(LayoutKind.Sequential)]
public struct PackedHalogenMaterial         // 84 B
{
    public uint materialID;
    public Vector4 albedo;
    public Vector4 specularAlbedo;
    public float metallic;
    public float roughness;
    public Vector4 emissive;                // (emission rgb, intensity)
    public PackedRayMedium rayMedium;
}

[StructLayout(LayoutKind.Sequential)]
public struct HalogenTriangle               // 72 B
{
    public Vector3 pointA, pointB, pointC;
    public Vector3 normalA, normalB, normalC;
}

[System.Serializable]
[StructLayout(LayoutKind.Sequential)]
public struct BVHEntry                      // 32 B; triangleCount > 0: leaf at indexA, else children indexA, indexA+1
{
    public uint indexA;
    public uint triangleCount;
    public Vector3 boundingCornerA;
    public Vector3 boundingCornerB;
}
