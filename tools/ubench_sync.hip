// Cost of cross-workgroup synchronisation on gfx950: one atomic per
// workgroup on a single address (u32), with and without a device-scope
// release fence before it; compared with an empty kernel.  Informs whether
// kernel boundaries can be replaced by last-workgroup tickets.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

template <int MODE>
__global__ __launch_bounds__(256) void k(unsigned* ctr, unsigned* out)
{
    __shared__ unsigned t;
    out[blockIdx.x * 256 + threadIdx.x] = threadIdx.x;  // a little dirty data per workgroup
    if (MODE == 0) return;
    __syncthreads();
    if (threadIdx.x == 0) {
        if (MODE == 2) __threadfence();
        if (MODE == 3) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        t = atomicAdd(ctr + (MODE == 4 ? (blockIdx.x & 31) * 32 : 0), 1u);
    }
    __syncthreads();
    if (MODE != 4 && t == gridDim.x - 1 && threadIdx.x == 0) { *ctr = 0; }
    if (MODE == 4 && threadIdx.x == 0 && t == gridDim.x / 32 - 1) ctr[(blockIdx.x & 31) * 32] = 0;
}

int main()
{
    unsigned *ctr, *out;
    CK(hipMalloc(&ctr, 4096 * 4));
    CK(hipMemset(ctr, 0, 4096 * 4));
    CK(hipMalloc(&out, 8192 * 256 * 4));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const char* names[] = {"empty", "atomic", "threadfence+atomic", "release fence+atomic", "atomic on 32 addrs"};
    for (int grid : {256, 1024, 2048, 8192}) {
        for (int mode = 0; mode < 5; ++mode) {
            std::vector<float> ts;
            for (int rep = 0; rep < 7; ++rep) {
                CK(hipEventRecord(a));
                for (int i = 0; i < 20; ++i) {
                    switch (mode) {
                        case 0: hipLaunchKernelGGL(k<0>, dim3(grid), dim3(256), 0, 0, ctr, out); break;
                        case 1: hipLaunchKernelGGL(k<1>, dim3(grid), dim3(256), 0, 0, ctr, out); break;
                        case 2: hipLaunchKernelGGL(k<2>, dim3(grid), dim3(256), 0, 0, ctr, out); break;
                        case 3: hipLaunchKernelGGL(k<3>, dim3(grid), dim3(256), 0, 0, ctr, out); break;
                        case 4: hipLaunchKernelGGL(k<4>, dim3(grid), dim3(256), 0, 0, ctr, out); break;
                    }
                }
                CK(hipEventRecord(b));
                CK(hipEventSynchronize(b));
                float ms;
                CK(hipEventElapsedTime(&ms, a, b));
                ts.push_back(ms * 1000 / 20);
            }
            std::sort(ts.begin(), ts.end());
            printf("grid %5d  %-22s %7.2f us per launch (back-to-back)\n", grid, names[mode], ts[3]);
        }
    }
    return 0;
}
