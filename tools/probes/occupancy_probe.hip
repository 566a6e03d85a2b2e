// Occupancy probe: how many waves of a workgroup shape actually run concurrently on one CU.
// Each workgroup's wave 0 registers itself in a per-CU counter (keyed by XCC/SE/SH/CU from the
// hardware id registers), records the running maximum, spins ~spin_us, and unregisters.
// build: hipcc --offload-arch=gfx950 -O2 tools/probes/occupancy_probe.hip -o build/occupancy_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

__global__ void probe(int* cnt, int* maxc, long long spin_cycles) {
    extern __shared__ int lds[];
    if (threadIdx.x % 64 == 0) {
        const unsigned hw = __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));    // HW_REG_HW_ID
        const unsigned xcc = __builtin_amdgcn_s_getreg((20) | (0 << 6) | (3 << 11));   // HW_REG_XCC_ID
        const unsigned cu = (hw >> 8) & 15, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
        const int id = (int)((((xcc & 15) * 8 + se) * 2 + sh) * 16 + cu);
        const int c = atomicAdd(&cnt[id], 1) + 1;
        atomicMax(&maxc[id], c);
        lds[threadIdx.x % 4] = c;
        const long long t0 = clock64();
        while (clock64() - t0 < spin_cycles) __builtin_amdgcn_s_sleep(2);
        atomicSub(&cnt[id], 1);
    }
}

int main(int argc, char** argv) {
    const int N = 16 * 8 * 2 * 16;
    int *cnt, *maxc;
    hipMalloc(&cnt, N * sizeof(int));
    hipMalloc(&maxc, N * sizeof(int));
    int ncu = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    const int shapes[][2] = {{64, 0}, {64, 10112}, {64, 11136}, {128, 0}, {256, 0}, {256, 38400}, {64, 4096}, {128, 20224}};
    for (auto& sh : shapes) {
        const int threads = sh[0], lds = sh[1];
        int occ = 0;
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, probe, threads, lds);
        hipMemset(cnt, 0, N * sizeof(int));
        hipMemset(maxc, 0, N * sizeof(int));
        const int blocks = ncu * 64;
        hipLaunchKernelGGL(probe, dim3(blocks), dim3(threads), lds, 0, cnt, maxc, 200000LL);
        hipDeviceSynchronize();
        int* h = (int*)malloc(N * sizeof(int));
        hipMemcpy(h, maxc, N * sizeof(int), hipMemcpyDeviceToHost);
        int mx = 0, mn = 1 << 30, used = 0;
        for (int i = 0; i < N; ++i)
            if (h[i]) { used++; mx = h[i] > mx ? h[i] : mx; mn = h[i] < mn ? h[i] : mn; }
        printf("threads %3d lds %6d: occupancy API %2d WG/CU; measured concurrent WG per CU max %d min %d over %d CUs\n",
               threads, lds, occ, mx, mn, used);
        free(h);
    }
    return 0;
}
