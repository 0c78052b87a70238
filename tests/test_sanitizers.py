"""Sanitizer builds of the native host code (SURVEY.md §5 "race detection / sanitizers"; GPU sanitizers are not
available on this pool, so the HIP kernels are covered by the bit-exact parity tests instead):

- the CPU oracle under AddressSanitizer + UndefinedBehaviorSanitizer (oracle/sanitize_main.c, make -C oracle
  sanitize), rendering golden cases on several pthreads: no report, and the image bit-identical to the regular
  oracle build's;
- the oracle's BVH builder (BVHGenerator.cs restated) under the same sanitizers;
- the product's parallel BLAS builder hg_build_blas_mt (std::thread pool, atomics; csrc/hg_host.cpp) under
  ThreadSanitizer (halogen-pathtracer_amd/host/tsan_blas.cpp, make -C halogen-pathtracer_amd tsan), large enough to
  take the rank-parallel partition, with 2, 5 and 16 workers: no data race, output equal to the sequential build."""
import os
import subprocess
from pathlib import Path

import numpy as np
import pytest

import cases
import hg_oracle
from halogen import host_files

ROOT = Path(__file__).resolve().parents[1]
ASAN = ROOT / "oracle" / "build" / "hg_oracle_asan"
TSAN = ROOT / "halogen-pathtracer_amd" / "build" / "tsan_blas"
ASAN_SAH = ROOT / "halogen-pathtracer_amd" / "build" / "asan_sah"
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
           UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1", TSAN_OPTIONS="halt_on_error=1:exitcode=66")


@pytest.fixture(scope="module")
def asan():
    subprocess.run(["make", "-s", "-C", str(ROOT / "oracle"), "sanitize"], check=True)
    return ASAN


@pytest.fixture(scope="module")
def tsan():
    subprocess.run(["make", "-s", "-C", str(ROOT / "halogen-pathtracer_amd"), "tsan"], check=True)
    return TSAN


def run(cmd):
    r = subprocess.run([str(c) for c in cmd], env=ENV, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and "Sanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-3000:]
    return r.stdout


@pytest.mark.parametrize("name", ["c1_64", "glass_64x36", "dragon1_64x36", "c1_32_tritests"])
def test_oracle_under_asan_ubsan(built, asan, tmp_path, name):
    packed, params, cube, frames, acc = cases.setup(name)
    host_files.write_scene(packed, tmp_path / "s.hgscene")
    (tmp_path / "p.bin").write_bytes(bytes(params))
    cmd = [asan, "render", tmp_path / "s.hgscene", tmp_path / "p.bin", frames, 3, tmp_path / "out.f32"]
    if cube is not None:
        host_files.write_cubemap(cube, tmp_path / "c.hgcube")
        cmd.append(tmp_path / "c.hgcube")
    run(cmd)
    W, H = int(params.screenParameters.x), int(params.screenParameters.y)
    got = np.fromfile(tmp_path / "out.f32", dtype=np.float32).reshape(H, W, 4)
    want, _ = hg_oracle.render(packed, params, frames, True, cubemap=cube)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))


def test_oracle_bvh_builder_under_asan_ubsan(asan):
    assert "BVH entries" in run([asan, "blas", 20000, 3])


def test_parallel_blas_builder_under_tsan(tsan):
    out = run([tsan, 40000, 7, 2, 5, 16])
    assert out.count("identical") == 3


POOL_DRIVER = r'''
#include "hg_host_pool.h"
#include <cstdio>
#include <vector>
int main() {
    std::vector<long> v(1000, 0);
    for (int rep = 0; rep < 500; ++rep)  // many back-to-back jobs: the generation / done hand-off between jobs
        HgHostPool::get().run(37, [&](size_t t) { for (size_t i = t; i < v.size(); i += 37) v[i] += 1; });
    long s = 0;
    for (long x : v) s += x;
    std::printf("%ld %d\n", s, HgHostPool::get().threads());
    return s == 500L * 1000 ? 0 : 1;
}
'''


def test_host_pool_under_tsan(tmp_path):
    """The persistent host pool of hg_upload_scene (csrc/hg_host_pool.h) under ThreadSanitizer: every task of every
    job runs exactly once, with no data race between jobs."""
    (tmp_path / "pool.cpp").write_text(POOL_DRIVER)
    exe = tmp_path / "pool"
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=thread",
                    f"-I{ROOT / 'halogen-pathtracer_amd' / 'csrc'}", str(tmp_path / "pool.cpp"), "-o", str(exe),
                    "-lpthread"], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "ThreadSanitizer" not in r.stderr, r.stderr[-2000:]
    assert r.stdout.split()[0] == str(500 * 1000)


def test_sah_builder_under_asan_ubsan():
    """hg_build_blas_sah (the non-reference SAH hierarchy, csrc/hg_host.cpp) under AddressSanitizer + UBSan: random
    soups, a flat grid (every box thin, padded), coincident triangles, an empty mesh, denormal and near-FLT_MAX
    coordinates (-fsanitize=float-cast-overflow: no bin conversion out of range); every triangle in one leaf; a NaN or
    infinite vertex rejected."""
    subprocess.run(["make", "-s", "-C", str(ROOT / "halogen-pathtracer_amd"), "asan_sah"], check=True)
    out = run([ASAN_SAH, 20000, 7])
    assert out.count("every triangle in one leaf") == 12, out
    assert out.count("non-finite vertex rejected") == 2, out
