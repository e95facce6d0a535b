// Micro-benchmark of single-wave primitive costs on gfx950 (development tool): cycles per iteration of
// dependent chains, measured with s_memtime inside one wave of a 512-thread block (7 waves idle at a barrier).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__global__ __launch_bounds__(512) void k(long long* out, int* g, int iters) {
    __shared__ int lds[4096];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int i = threadIdx.x; i < 4096; i += 512) lds[i] = (i * 7 + 1) & 4095;
    __syncthreads();
    if (wave == 0) {
        long long t0, t1;
        int x = lane;
        // 1. dependent ds_read chain
        t0 = __builtin_amdgcn_s_memtime();
        for (int i = 0; i < iters; i++) x = lds[x];
        t1 = __builtin_amdgcn_s_memtime();
        if (lane == 0) out[0] = t1 - t0;
        // 2. ballot + ffs + readlane chain (uniform)
        int y = x & 63;
        t0 = __builtin_amdgcn_s_memtime();
        for (int i = 0; i < iters; i++) {
            uint64_t m = __ballot(((lane ^ y) & 3) == 0);
            y = (__builtin_amdgcn_readlane(x + i, (__ffsll((unsigned long long)m) - 1 + y) & 63)) & 63;
        }
        t1 = __builtin_amdgcn_s_memtime();
        if (lane == 0) out[1] = t1 - t0;
        // 3. VALU chain (64-bit compare/select)
        int64_t z = x;
        t0 = __builtin_amdgcn_s_memtime();
        for (int i = 0; i < iters; i++) z = (z > (int64_t)i) ? z - i : z + 3;
        t1 = __builtin_amdgcn_s_memtime();
        if (lane == 0) out[2] = t1 - t0;
        // 4. single-lane global store per iteration
        t0 = __builtin_amdgcn_s_memtime();
        for (int i = 0; i < iters; i++)
            if (lane == 0) g[(i * 64) & 0xFFFF] = i + (int)z;
        t1 = __builtin_amdgcn_s_memtime();
        if (lane == 0) out[3] = t1 - t0;
        // 5. shfl_down chain
        int w = x;
        t0 = __builtin_amdgcn_s_memtime();
        for (int i = 0; i < iters; i++) w = __shfl_down(w, 1) + 1;
        t1 = __builtin_amdgcn_s_memtime();
        if (lane == 0) out[4] = t1 - t0;
        // 6. atomicAdd (no return) on 4 lanes
        t0 = __builtin_amdgcn_s_memtime();
        for (int i = 0; i < iters; i++)
            if (lane < 4) atomicAdd((unsigned long long*)&g[70000 + 2 * lane], 1ull);
        t1 = __builtin_amdgcn_s_memtime();
        if (lane == 0) out[5] = t1 - t0;
        // 7. empty uniform loop with s_memtime (clock overhead)
        long long acc = 0;
        t0 = __builtin_amdgcn_s_memtime();
        for (int i = 0; i < iters; i++) acc += __builtin_amdgcn_s_memtime();
        t1 = __builtin_amdgcn_s_memtime();
        if (lane == 0) out[6] = t1 - t0 + (acc & 1);
        if (lane == 0) out[7] = x + y + w + (int)z;
    }
}

int main() {
    long long* out;
    int* g;
    hipMalloc(&out, 8 * sizeof(long long));
    hipMalloc(&g, 80000 * sizeof(int));
    hipMemset(g, 0, 80000 * sizeof(int));
    const int iters = 4096;
    for (int rep = 0; rep < 2; rep++) {
        hipLaunchKernelGGL(k, dim3(1), dim3(512), 0, 0, out, g, iters);
        hipDeviceSynchronize();
    }
    long long h[8];
    hipMemcpy(h, out, sizeof h, hipMemcpyDeviceToHost);
    const char* names[7] = {"ds_read chain", "ballot+ffs+readlane chain", "valu int64 select chain", "1-lane global store",
                            "shfl_down chain", "4-lane atomicAdd", "s_memtime"};
    for (int i = 0; i < 7; i++) printf("%-28s %8.1f cycles/iter\n", names[i], (double)h[i] / iters);
    return 0;
}
