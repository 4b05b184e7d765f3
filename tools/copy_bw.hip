// Diagnostic: the HBM copy ceiling K0's speculative stored copy runs against (C4 noise).
// 1 GiB in -> 1 GiB out, the access shapes K0 uses (one workgroup per 32 KiB block, 8
// independent 16 B loads per lane, then 8 stores) and some others, timed with HIP events.
// Reports (read + write) bytes / time.
// build: hipcc -O3 --offload-arch=gfx950 -o tools/copy_bw tools/copy_bw.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

// one workgroup per block of 256 * 16 * U bytes: U loads per lane in flight, then U stores
template <int U, bool NT>
__global__ __launch_bounds__(256) void blk_copy(const uint4* __restrict__ in, uint4* __restrict__ out) {
    const uint64_t base = (uint64_t)blockIdx.x * 256 * U + threadIdx.x;
    uint4 v[U];
#pragma unroll
    for (int k = 0; k < U; k++) v[k] = in[base + 256 * k];
#pragma unroll
    for (int k = 0; k < U; k++) {
        if (NT) {
            typedef uint32_t u4v __attribute__((ext_vector_type(4)));
            const u4v x = {v[k].x, v[k].y, v[k].z, v[k].w};
            __builtin_nontemporal_store(x, reinterpret_cast<u4v*>(&out[base + 256 * k]));
        } else {
            out[base + 256 * k] = v[k];
        }
    }
}

// grid-stride: U loads per lane per trip
template <int U>
__global__ __launch_bounds__(256) void gs_copy(const uint4* __restrict__ in, uint4* __restrict__ out, uint64_t n16) {
    const uint64_t stride = (uint64_t)gridDim.x * 256 * U;
    for (uint64_t b = (uint64_t)blockIdx.x * 256 * U + threadIdx.x; b < n16; b += stride) {
        uint4 v[U];
#pragma unroll
        for (int k = 0; k < U; k++) v[k] = in[b + 256 * k];
#pragma unroll
        for (int k = 0; k < U; k++) out[b + 256 * k] = v[k];
    }
}

template <int U>
__global__ __launch_bounds__(256) void blk_read(const uint4* __restrict__ in, uint32_t* __restrict__ sink) {
    const uint64_t base = (uint64_t)blockIdx.x * 256 * U + threadIdx.x;
    uint32_t x = 0;
#pragma unroll
    for (int k = 0; k < U; k++) {
        const uint4 v = in[base + 256 * k];
        x ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (x == 0x12345678u) sink[0] = x;
}

template <int U>
__global__ __launch_bounds__(256) void blk_write(uint4* __restrict__ out) {
    const uint64_t base = (uint64_t)blockIdx.x * 256 * U + threadIdx.x;
#pragma unroll
    for (int k = 0; k < U; k++) out[base + 256 * k] = make_uint4(k, 1, 2, 3);
}

int main() {
    const uint64_t n = 1ull << 30, n16 = n / 16;
    uint4 *in, *out;
    uint32_t* sink;
    CK(hipMalloc(&in, n));
    CK(hipMalloc(&out, n));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(in, 0x5A, n));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run = [&](const char* name, double bytes, auto launch) -> int {
        for (int w = 0; w < 3; w++) launch();
        CK(hipDeviceSynchronize());
        const int R = 20;
        CK(hipEventRecord(e0));
        for (int r = 0; r < R; r++) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double t = ms / R;
        printf("%-36s %8.4f ms  %7.3f TB/s\n", name, t, bytes / (t * 1e-3) / 1e12);
        return 0;
    };
    const double rw = 2.0 * n;
    run("blk_copy<8> (K0 shape, 32 KiB/WG)", rw, [&] { hipLaunchKernelGGL((blk_copy<8, false>), dim3(n16 / 2048), dim3(256), 0, 0, in, out); });
    run("blk_copy<8> nontemporal stores", rw, [&] { hipLaunchKernelGGL((blk_copy<8, true>), dim3(n16 / 2048), dim3(256), 0, 0, in, out); });
    run("blk_copy<4> (16 KiB/WG)", rw, [&] { hipLaunchKernelGGL((blk_copy<4, false>), dim3(n16 / 1024), dim3(256), 0, 0, in, out); });
    run("blk_copy<16> (64 KiB/WG)", rw, [&] { hipLaunchKernelGGL((blk_copy<16, false>), dim3(n16 / 4096), dim3(256), 0, 0, in, out); });
    run("gs_copy<4> 2048 WGs", rw, [&] { hipLaunchKernelGGL((gs_copy<4>), dim3(2048), dim3(256), 0, 0, in, out, n16); });
    run("gs_copy<8> 4096 WGs", rw, [&] { hipLaunchKernelGGL((gs_copy<8>), dim3(4096), dim3(256), 0, 0, in, out, n16); });
    run("hipMemcpyDtoD", rw, [&] { (void)hipMemcpyAsync(out, in, n, hipMemcpyDeviceToDevice, 0); });
    run("blk_read<8> (read only)", (double)n, [&] { hipLaunchKernelGGL((blk_read<8>), dim3(n16 / 2048), dim3(256), 0, 0, in, sink); });
    run("blk_write<8> (write only)", (double)n, [&] { hipLaunchKernelGGL((blk_write<8>), dim3(n16 / 2048), dim3(256), 0, 0, out); });
    return 0;
}
