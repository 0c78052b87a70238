"""Stand-ins for the UnityEngine pieces the reference's host side leans on.

The reference runs inside Unity 2022.3 (ProjectSettings/ProjectVersion.txt:1); its buffers are built from
Unity transforms (Transform.localToWorldMatrix / worldToLocalMatrix), Unity's built-in Plane and Cube
meshes (engine assets, not in the repository) and UnityEngine.Bounds.  None of that exists here, so this
module DEFINES deterministic equivalents (documented in DESIGN.md §scene).  They are inputs: the GPU path
and the CPU oracle consume the same packed arrays, so parity does not depend on matching Unity's exact bits.
"""
from __future__ import annotations

import math

import numpy as np

f32 = np.float32


def quat_to_mat3(q) -> np.ndarray:
    """Unit quaternion (x, y, z, w) -> 3x3 rotation (Unity's Matrix4x4.Rotate formula), float64."""
    x, y, z, w = (float(v) for v in q)
    n = math.sqrt(x * x + y * y + z * z + w * w)
    x, y, z, w = x / n, y / n, z / n, w / n
    return np.array([
        [1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
        [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
        [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)],
    ], dtype=np.float64)


def quat_mul(a, b) -> np.ndarray:
    """Hamilton product a * b of quaternions (x, y, z, w), float64 (Unity's Quaternion * Quaternion)."""
    ax, ay, az, aw = (float(v) for v in a)
    bx, by, bz, bw = (float(v) for v in b)
    return np.array([aw * bx + ax * bw + ay * bz - az * by,
                     aw * by + ay * bw + az * bx - ax * bz,
                     aw * bz + az * bw + ax * by - ay * bx,
                     aw * bw - ax * bx - ay * by - az * bz], dtype=np.float64)


def euler_to_quat(ex: float, ey: float, ez: float):
    """Unity Euler angles in degrees (applied Z, then X, then Y) -> quaternion (x, y, z, w)."""
    def axis(ax, deg):
        h = math.radians(deg) * 0.5
        s = math.sin(h)
        return np.array([ax[0] * s, ax[1] * s, ax[2] * s, math.cos(h)])

    def mul(a, b):
        ax, ay, az, aw = a
        bx, by, bz, bw = b
        return np.array([aw * bx + ax * bw + ay * bz - az * by, aw * by - ax * bz + ay * bw + az * bx,
                         aw * bz + ax * by - ay * bx + az * bw, aw * bw - ax * bx - ay * by - az * bz])

    q = mul(mul(axis((0, 1, 0), ey), axis((1, 0, 0), ex)), axis((0, 0, 1), ez))
    return tuple(q)


def trs(pos, rot_quat, scale) -> np.ndarray:
    """Matrix4x4.TRS as a 4x4 float64 (row r, column c)."""
    m = np.eye(4)
    m[:3, :3] = quat_to_mat3(rot_quat) * np.asarray(scale, dtype=np.float64)[None, :]
    m[:3, 3] = np.asarray(pos, dtype=np.float64)
    return m


def to_unity_floats(m: np.ndarray) -> list[float]:
    """4x4 (row, col) -> the 16 floats of UnityEngine.Matrix4x4 in field order m00, m10, m20, m30, m01 ..."""
    return [float(f32(v)) for v in np.asarray(m, dtype=np.float64).T.reshape(-1)]


class Transform:
    """A Unity Transform with an optional parent; matrices in float64, rounded to float32 when packed."""

    def __init__(self, position=(0, 0, 0), rotation=(0, 0, 0, 1), scale=(1, 1, 1), parent: "Transform | None" = None):
        self.position_local = tuple(float(v) for v in position)
        self.rotation_local = tuple(float(v) for v in rotation)
        self.scale_local = tuple(float(v) for v in scale)
        self.parent = parent

    @property
    def local_to_world(self) -> np.ndarray:
        m = trs(self.position_local, self.rotation_local, self.scale_local)
        return m if self.parent is None else self.parent.local_to_world @ m

    @property
    def world_to_local(self) -> np.ndarray:
        return np.linalg.inv(self.local_to_world)

    @property
    def position(self) -> np.ndarray:
        """World position as float32 (Transform.position)."""
        return self.local_to_world[:3, 3].astype(np.float32)

    @property
    def rotation(self) -> np.ndarray:
        """World rotation (x, y, z, w) as float32 (Transform.rotation = parent.rotation * localRotation); scale plays
        no part in it."""
        q = np.asarray(self.rotation_local, dtype=np.float64)
        q = q / math.sqrt(float(q @ q))
        if self.parent is not None:
            q = quat_mul(self.parent.rotation.astype(np.float64), q)
        return q.astype(np.float32)


# -------------------------------------------------------------------------------------------------
# Built-in primitive meshes (engine assets in Unity; regenerated here).  Triangles are wound so that
# cross(v1 - v0, v2 - v0) is the outward normal, i.e. a ray from outside hits with orientation +1.
# -------------------------------------------------------------------------------------------------
def unity_plane():
    """Unity's built-in Plane: 10 x 10 units in XZ, 11 x 11 vertices, 200 triangles, normal +Y."""
    xs = np.arange(11, dtype=np.float32) - f32(5)
    verts, norms = [], []
    for iz in range(11):
        for ix in range(11):
            verts.append((xs[ix], 0.0, xs[iz]))
            norms.append((0.0, 1.0, 0.0))
    idx = []
    for iz in range(10):
        for ix in range(10):
            v00 = iz * 11 + ix
            v10, v01 = v00 + 1, v00 + 11
            v11 = v01 + 1
            idx.append((v00, v01, v11))
            idx.append((v00, v11, v10))
    return (np.array(verts, dtype=np.float32), np.array(norms, dtype=np.float32), np.array(idx, dtype=np.int32))


def unity_cube():
    """Unity's built-in Cube: unit cube centred at the origin, 24 vertices (4 per face), 12 triangles."""
    faces = [  # (normal, u, v) with u x v = normal
        ((1, 0, 0), (0, 1, 0), (0, 0, 1)), ((-1, 0, 0), (0, 0, 1), (0, 1, 0)),
        ((0, 1, 0), (0, 0, 1), (1, 0, 0)), ((0, -1, 0), (1, 0, 0), (0, 0, 1)),
        ((0, 0, 1), (1, 0, 0), (0, 1, 0)), ((0, 0, -1), (0, 1, 0), (1, 0, 0)),
    ]
    verts, norms, idx = [], [], []
    for n, u, v in faces:
        n, u, v = (np.array(a, dtype=np.float64) for a in (n, u, v))
        base = len(verts)
        for a, b in ((-0.5, -0.5), (0.5, -0.5), (0.5, 0.5), (-0.5, 0.5)):
            verts.append(n * 0.5 + u * a + v * b)
            norms.append(n)
        idx.append((base, base + 1, base + 2))
        idx.append((base, base + 2, base + 3))
    return (np.array(verts, dtype=np.float32), np.array(norms, dtype=np.float32), np.array(idx, dtype=np.int32))


def mesh_bounds_min_max(verts: np.ndarray):
    """Raw vertex extremes (the input of Unity's mesh.bounds = Bounds.SetMinMax(min, max))."""
    return verts.min(axis=0).astype(np.float32), verts.max(axis=0).astype(np.float32)
