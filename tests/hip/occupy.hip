// Test-only helper (not part of the product library): a kernel that holds CUs for a bounded time, so a test can
// force a co-residency failure of the grouped LSTM (csrc/lstm_group.hip).  Each workgroup takes the dynamic LDS it
// is launched with (160 KB: one workgroup per CU, and no 136 KB LSTM workgroup fits beside it), counts itself into
// *arrived (a vector atomic on global memory), and sleeps until `ticks` of the 100 MHz realtime counter have passed.
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ void occupy_kernel(unsigned* arrived, uint64_t ticks) {
    extern __shared__ float lds[];
    if (threadIdx.x == 0) atomicAdd(arrived, 1u);
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(127);
    lds[threadIdx.x] = 0.f;
}

extern "C" int occupy_cus(int nblocks, unsigned* arrived, double seconds, void* stream) {
    const size_t lds = 160 * 1024;
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(&occupy_kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)lds) != hipSuccess)
        return -1;
    if (seconds <= 0 || seconds > 10) return -2;                       // bounded by construction
    hipLaunchKernelGGL(occupy_kernel, dim3(nblocks), dim3(64), lds, (hipStream_t)stream, arrived,
                       (uint64_t)(seconds * 1e8));
    return hipGetLastError() == hipSuccess ? 0 : -3;
}
