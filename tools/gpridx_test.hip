// Diagnostic: does s_set_gpr_idx_on (SRC0) index the VGPR source of v_readlane_b32 on gfx950?
// Each of v96..v111 holds 1000 * reg + lane; reads lane `ln` of register 96 + idx with the index
// mode on, straight into an SGPR.  Prints OK when every (idx, ln) gives 1000 * idx + ln.
#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void k(unsigned* out) {
    const unsigned lane = threadIdx.x;
    unsigned bad = 0;
    for (unsigned idx = 0; idx < 16; idx++) {
        for (unsigned ln = 0; ln < 64; ln += 7) {
            unsigned r;
            asm volatile(
                "v_mov_b32 v96, %[l]\n v_add_u32 v97, 1000, %[l]\n v_add_u32 v98, 2000, %[l]\n v_add_u32 v99, 3000, %[l]\n"
                "v_add_u32 v100, 4000, %[l]\n v_add_u32 v101, 5000, %[l]\n v_add_u32 v102, 6000, %[l]\n v_add_u32 v103, 7000, %[l]\n"
                "v_add_u32 v104, 8000, %[l]\n v_add_u32 v105, 9000, %[l]\n v_add_u32 v106, 10000, %[l]\n v_add_u32 v107, 11000, %[l]\n"
                "v_add_u32 v108, 12000, %[l]\n v_add_u32 v109, 13000, %[l]\n v_add_u32 v110, 14000, %[l]\n v_add_u32 v111, 15000, %[l]\n"
                "s_mov_b32 s89, m0\n"
                "s_nop 4\n"
                "s_set_gpr_idx_on %[i], gpr_idx(SRC0)\n"
                "v_readlane_b32 %[r], v96, %[n]\n"
                "s_set_gpr_idx_off\n"
                "s_mov_b32 m0, s89\n"
                : [r] "=s"(r) : [l] "v"(lane), [i] "s"(idx), [n] "s"(ln)
                : "s89", "v96", "v97", "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107",
                  "v108", "v109", "v110", "v111");
            if (r != 1000 * idx + ln) bad++;
        }
    }
    if (lane == 0) out[0] = bad;
}
int main() {
    unsigned* d; unsigned h = 12345;
    hipMalloc(&d, 4);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    hipMemcpy(&h, d, 4, hipMemcpyDeviceToHost);
    printf("%s (%u mismatches)\n", h == 0 ? "OK" : "DIFFERENT", h);
    hipFree(d);
    return 0;
}
