// Diagnostic: the VALU issue ceiling of one MI355X for the roofline in bench.py.
// Independent 32-bit integer VALU instructions (v_add_u32 / v_xor_b32 / v_min_u32, the
// kind the match kernel issues), 8 independent chains per lane, no memory traffic.
// Reports wave64 VALU instructions per second for the whole chip and per SIMD cycle at the
// clock measured inside the kernel (s_memtime / s_memrealtime, 100 MHz reference), for
// 1, 2, 4 and 8 waves per SIMD.  Also a dependent DPP chain (one wave_shr per step) to
// show the latency a single chain pays.
// build: hipcc -O3 --offload-arch=gfx950 -o tools/valu_peak tools/valu_peak.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define ITERS 2048
#define PER_ITER 64   // VALU instructions in one asm block

template <int DPP>
__global__ void valu_kernel(uint32_t* out, unsigned long long* clk, uint32_t seed) {
    uint32_t a0 = seed + threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 11, a5 = a0 * 13, a6 = a0 * 17,
             a7 = a0 * 19;
    const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < ITERS; it++) {
        if (DPP == 2) {
            // 8 independent chains of single-instruction DPP moves (bound_ctrl: no old value)
#pragma unroll
            for (int k = 0; k < PER_ITER / 8; k++) {
                a0 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)a0, 0x138, 0xF, 0xF, true);
                a1 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)a1, 0x138, 0xF, 0xF, true);
                a2 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)a2, 0x138, 0xF, 0xF, true);
                a3 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)a3, 0x138, 0xF, 0xF, true);
                a4 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)a4, 0x138, 0xF, 0xF, true);
                a5 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)a5, 0x138, 0xF, 0xF, true);
                a6 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)a6, 0x138, 0xF, 0xF, true);
                a7 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)a7, 0x138, 0xF, 0xF, true);
            }
        } else if (DPP) {
            // 64 dependent DPP moves on one register (latency-bound chain)
#pragma unroll
            for (int k = 0; k < PER_ITER; k++)
                a0 = (uint32_t)__builtin_amdgcn_update_dpp((int)a1, (int)a0, 0x138, 0xF, 0xF, false);
        } else {
            asm volatile(
                ".rept 8\n"
                "v_add_u32 %0, %0, %1\n v_xor_b32 %1, %1, %2\n v_add_u32 %2, %2, %3\n v_xor_b32 %3, %3, %4\n"
                "v_add_u32 %4, %4, %5\n v_xor_b32 %5, %5, %6\n v_min_u32 %6, %6, %7\n v_add_u32 %7, %7, %0\n"
                ".endr\n"
                : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        clk[0] = t1 - t0;
        clk[1] = r1 - r0;
    }
    if ((a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7) == 0x12345u) out[0] = 1;
}

int main() {
    uint32_t* d;
    unsigned long long* dc;
    (void)hipMalloc(&d, 64);
    (void)hipMalloc(&dc, 64);
    hipDeviceProp_t p;
    (void)hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    printf("CUs %d\n", cus);
    for (int dpp = 0; dpp < 3; dpp++) {
        for (int wps = 1; wps <= 8; wps *= 2) {   // waves per SIMD: 256-thread workgroups, wps per CU
            const int blocks = cus * wps, threads = 256;
            for (int rep = 0; rep < 3; rep++) {
                (void)hipEventRecord(e0, 0);
                if (dpp == 2) hipLaunchKernelGGL(valu_kernel<2>, dim3(blocks), dim3(threads), 0, 0, d, dc, 7u);
                else if (dpp) hipLaunchKernelGGL(valu_kernel<1>, dim3(blocks), dim3(threads), 0, 0, d, dc, 7u);
                else hipLaunchKernelGGL(valu_kernel<0>, dim3(blocks), dim3(threads), 0, 0, d, dc, 7u);
                (void)hipEventRecord(e1, 0);
                (void)hipEventSynchronize(e1);
                if (rep < 2) continue;
                float ms = 0;
                (void)hipEventElapsedTime(&ms, e0, e1);
                unsigned long long hc[2];
                (void)hipMemcpy(hc, dc, 16, hipMemcpyDeviceToHost);
                const double ghz = hc[1] ? (double)hc[0] / (double)hc[1] * 0.1 : 0.0;
                const double winst = (double)blocks * (threads / 64) * ITERS * PER_ITER;
                const double rate = winst / (ms * 1e-3);
                const double per_simd_cycle = rate / (cus * 4.0) / (ghz * 1e9);
                printf("%s waves/SIMD %d: %.1f G wave-instr/s, in-kernel clock %.2f GHz, %.3f instr per SIMD cycle"
                       " (%.2f cycles per instr)\n",
                       dpp == 2 ? "8 independent DPP    " : dpp ? "dependent DPP chain  " : "independent int VALU ", wps, rate * 1e-9, ghz, per_simd_cycle,
                       1.0 / per_simd_cycle);
            }
        }
    }
    return 0;
}
