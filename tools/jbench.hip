// Diagnostic microbenchmark of the match kernel's candidate step (DPP shift + 16-byte compare).
// 1024-thread workgroups (16 waves), one per CU; reports cycles per step per wave.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#define STEPS 4096
__device__ __forceinline__ uint32_t wshr(uint32_t v, uint32_t lane0) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)lane0, (int)v, 0x138, 0xF, 0xF, false);
}
__device__ __forceinline__ uint32_t mb(uint64_t x) { return x ? ((uint32_t)__builtin_ctzll(x) >> 3) : 8u; }
template <int V>
__global__ __launch_bounds__(1024) void k(unsigned long long* out, uint32_t seed) {
    const uint32_t lane = threadIdx.x & 63;
    uint32_t h0 = seed * lane + 1, h1 = h0 * 3, h2 = h0 * 5, h3 = h0 * 7, hq = lane * 11;
    uint32_t x0l = h0 ^ 0x55, x0h = h1, x1l = h2, x1h = h3, xq = hq;
    uint64_t iv0 = ((uint64_t)h1 << 32) | h0, iv1 = ((uint64_t)h3 << 32) | h2;
    uint32_t best = 0, lim = 200, nc = 20;
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (uint32_t j = 1; j <= STEPS; j++) {
        const int src = (int)(j & 31);
        if (V == 0 || V == 1 || V == 3) {
            xq = wshr(xq, __builtin_amdgcn_readlane(hq, src));
            x0l = wshr(x0l, __builtin_amdgcn_readlane(h0, src));
            x0h = wshr(x0h, __builtin_amdgcn_readlane(h1, src));
            x1l = wshr(x1l, __builtin_amdgcn_readlane(h2, src));
            x1h = wshr(x1h, __builtin_amdgcn_readlane(h3, src));
        } else {   // V == 2: no cross-lane: plain register rotation
            xq += 1; x0l ^= x0h; x0h += 3; x1l ^= xq; x1h += x1l;
        }
        if (V == 3) continue;   // shifts only
        const uint32_t m0 = mb(iv0 ^ (((uint64_t)x0h << 32) | x0l));
        uint32_t m = m0;
        if (V != 1) { const uint32_t m1 = mb(iv1 ^ (((uint64_t)x1h << 32) | x1l)); m = m0 < 8 ? m0 : 8 + m1; }
        m = min(m, lim);
        const uint32_t key = ((j & 31) <= nc && m >= 3) ? ((m << 15) | xq) : 0u;
        best = max(best, key);
    }
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) atomicAdd(out, (unsigned long long)((t1 - t0) / STEPS));
    if (best == 0x7777 && xq == 3) out[1] = best + x0l + x1h;
}
int main() {
    unsigned long long* d;
    (void)hipMalloc(&d, 64);
    const char* nm[] = {"full step (5 shifts + 16B compare)", "5 shifts + 8B compare", "no DPP (register ops) + 16B compare", "5 shifts only"};
    for (int v = 0; v < 4; v++) {
        for (int rep = 0; rep < 2; rep++) {
            (void)hipMemset(d, 0, 64);
            void (*f)(unsigned long long*, uint32_t) = v == 0 ? k<0> : v == 1 ? k<1> : v == 2 ? k<2> : k<3>;
            hipLaunchKernelGGL(f, dim3(256), dim3(1024), 0, 0, d, 7u);
            (void)hipDeviceSynchronize();
            unsigned long long h;
            (void)hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
            if (rep) printf("%-40s %7.1f cycles per step per wave (16 waves/CU)\n", nm[v], h / 4096.0);
        }
    }
    return 0;
}
