// Diagnostic: are LDS atomicAdd return values for same-address lanes of ONE wave
// instruction ordered by lane on gfx950?  Prints violations over many random patterns.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
__global__ __launch_bounds__(1024) void k(uint32_t seed, uint32_t* viol, uint32_t* checks, int mode) {
    __shared__ uint32_t C[16 * 128];
    for (int t = threadIdx.x; t < 16 * 128; t += 1024) C[t] = 0;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t x = seed * 2654435761u + threadIdx.x * 40503u + blockIdx.x * 977u;
    uint32_t bad = 0, chk = 0;
    for (int st = 0; st < 64; st++) {
        x = x * 1664525u + 1013904223u;
        uint32_t d = mode == 0 ? (x >> 25) : mode == 1 ? ((x >> 28) & 3) : (mode == 2 ? 5u : ((x >> 20) & 127) % (1 + (st & 7)));
        const uint32_t r = atomicAdd(&C[wave * 128 + d], 1u);
        // compare with every earlier lane of the same digit (via LDS exchange of (d, r))
        __shared__ uint32_t D[1024], Rr[1024];
        D[threadIdx.x] = d; Rr[threadIdx.x] = r;
        __syncthreads();
        for (uint32_t l2 = 0; l2 < lane; l2++) {
            const uint32_t t2 = wave * 64 + l2;
            if (D[t2] == d) { chk++; if (Rr[t2] > r) bad++; }
        }
        __syncthreads();
    }
    atomicAdd(viol, bad);
    atomicAdd(checks, chk);
}
int main() {
    uint32_t *v, *c;
    (void)hipMalloc(&v, 8); (void)hipMalloc(&c, 8);
    for (int mode = 0; mode < 4; mode++) {
        (void)hipMemset(v, 0, 8); (void)hipMemset(c, 0, 8);
        for (int rep = 0; rep < 50; rep++) hipLaunchKernelGGL(k, dim3(1024), dim3(1024), 0, 0, (uint32_t)rep, v, c, mode);
        (void)hipDeviceSynchronize();
        uint32_t hv, hc; (void)hipMemcpy(&hv, v, 4, hipMemcpyDeviceToHost); (void)hipMemcpy(&hc, c, 4, hipMemcpyDeviceToHost);
        printf("mode %d: %u same-address lane pairs checked, %u out of lane order\n", mode, hc, hv);
    }
    return 0;
}
