// LDS read-cost microbenchmark (diagnostic): 1024-thread WG, 16 waves, 64 KiB LDS,
// each lane does N dependent-address reads of one flavour; reports cycles per wave-read.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#define N 2048
template <int MODE>
__global__ __launch_bounds__(1024) void k(unsigned long long* out, uint32_t seed, int rnd) {
    __shared__ uint32_t lds[16384];
    for (int i = threadIdx.x; i < 16384; i++) lds[i] = i * 2654435761u + seed;
    __syncthreads();
    uint32_t x = threadIdx.x * 7 + seed, acc = 0;
    const uint8_t* b = (const uint8_t*)lds;
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < N; it++) {
        uint32_t a = rnd ? ((x * 2654435761u) >> 16) & 0xFFF0 : (threadIdx.x * 4 + it * 64) & 0xFFF0;
        if (MODE == 0) { acc += lds[a >> 2]; }                                     // aligned b32
        if (MODE == 1) { uint32_t v; __builtin_memcpy(&v, b + a + 1, 4); acc += v; } // unaligned b32
        if (MODE == 2) { uint64_t v = *(const uint64_t*)(b + a); acc += (uint32_t)v ^ (uint32_t)(v >> 32); } // aligned b64
        if (MODE == 3) { uint64_t v; __builtin_memcpy(&v, b + a + 3, 8); acc += (uint32_t)v ^ (uint32_t)(v >> 32); } // unaligned b64
        if (MODE == 4) { acc += b[a + 3]; }                                         // u8
        if (MODE == 5) { uint32_t w0 = lds[a >> 2], w1 = lds[(a >> 2) + 1]; acc += __builtin_amdgcn_alignbyte(w1, w0, 3); } // 2x b32 + alignbyte
        if (MODE == 6) { uint64_t v0 = *(const uint64_t*)(b + a), v1 = *(const uint64_t*)(b + a + 8);  // 2 aligned b64 + funnel
                         acc += (uint32_t)((v0 >> 24) | (v1 << 40)); }
        x = x * 1664525u + 1013904223u + acc;   // dependent next address
    }
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x & 63) == 0) atomicAdd(&out[0], (unsigned long long)((t1 - t0) / N));
    if (acc == 0x12345) out[1] = acc;
}
int main() {
    unsigned long long* d; (void)hipMalloc(&d, 64);
    const char* names[] = {"b32 aligned", "b32 unaligned", "b64 aligned", "b64 unaligned", "u8", "2xb32+alignbyte", "2xb64 aligned+funnel"};
    for (int rnd = 0; rnd < 2; rnd++)
    for (int m = 0; m < 7; m++) {
        for (int rep = 0; rep < 2; rep++) {
            (void)hipMemset(d, 0, 64);
            void (*f)(unsigned long long*, uint32_t, int) = m==0?k<0>:m==1?k<1>:m==2?k<2>:m==3?k<3>:m==4?k<4>:m==5?k<5>:k<6>;
            hipLaunchKernelGGL(f, dim3(256), dim3(1024), 0, 0, d, 1u, rnd);
            hipDeviceSynchronize();
            unsigned long long h[2]; hipError_t e = hipDeviceSynchronize(); (void)hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
            if (rep) printf("%-22s %s: %6.1f cycles per wave-iteration (avg over 16 waves)\n", names[m], rnd ? "random" : "contig", h[0] / 4096.0); if (e) printf("err %d\n", e);
        }
    }
    return 0;
}
