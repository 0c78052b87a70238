// hg_selftest.hip — device self-tests of arithmetic shortcuts the kernels rely on (hg_selftest in the C-ABI).
#include <hip/hip_runtime.h>

#include <cstdint>

// ---------------------------------------------------------------------------------------------------------
// self-test: the fast reciprocal path against IEEE division for all 2^32 inputs of its range
// ---------------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void hg_selftest_rcp_kernel(unsigned long long* mismatches, unsigned long long* tested) {
    unsigned long long bad = 0, cnt = 0;
    for (uint64_t u = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; u < (1ull << 32);
         u += uint64_t(gridDim.x) * blockDim.x) {
        const float x = __uint_as_float(uint32_t(u));
        const uint32_t ex = (uint32_t(u) >> 23) & 0xFFu;
        if (ex - 2u > 250u) continue;
        const float r = __builtin_amdgcn_rcpf(x);
        const float e = __builtin_fmaf(-x, r, 1.0f);
        const float fast = __builtin_fmaf(e, r, r);
        const float ref = 1.0f / x;
        bad += __float_as_uint(fast) != __float_as_uint(ref);
        cnt++;
    }
    atomicAdd(mismatches, bad);
    atomicAdd(tested, cnt);
}

int64_t hg_selftest_rcp_all(int64_t* tested) {
    unsigned long long* d = nullptr;
    if (hipMalloc(&d, 2 * sizeof(unsigned long long)) != hipSuccess) return -1;
    if (hipMemset(d, 0, 2 * sizeof(unsigned long long)) != hipSuccess) return -1;
    hipLaunchKernelGGL(hg_selftest_rcp_kernel, dim3(8192), dim3(256), 0, 0, d, d + 1);
    unsigned long long h[2] = {0, 0};
    if (hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return -1;
    (void)hipFree(d);
    if (tested) *tested = int64_t(h[1]);
    return int64_t(h[0]);
}
