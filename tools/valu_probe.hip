// VALU issue-rate probe: cycles per wave64 instruction per SIMD for the integer ops the
// rollout kernel is made of (v_lshl_or_b32, v_and_b32, v_bitop3_b32) vs v_fma_f32, at
// 1..8 waves per SIMD.  Used to fix the compute roofline's peak.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define N_ITERS 4096

template <int KIND>
__global__ __launch_bounds__(1024) void probe(uint32_t* out, uint32_t seed) {
    uint32_t a0 = seed ^ threadIdx.x, a1 = a0 * 3u, a2 = a0 * 5u, a3 = a0 * 7u, a4 = a0 * 11u, a5 = a0 * 13u,
             a6 = a0 * 17u, a7 = a0 * 19u;
    float f0 = (float)a0, f1 = f0 + 1.f, f2 = f0 + 2.f, f3 = f0 + 3.f, f4 = f0 + 4.f, f5 = f0 + 5.f, f6 = f0 + 6.f,
          f7 = f0 + 7.f;
    const uint32_t s = seed & 7u;
    for (int i = 0; i < N_ITERS; ++i) {
        if constexpr (KIND == 0) {  // 8 independent v_lshl_or_b32 per iteration
            asm volatile(
                "v_lshl_or_b32 %0, %1, %8, %0\n v_lshl_or_b32 %1, %2, %8, %1\n"
                "v_lshl_or_b32 %2, %3, %8, %2\n v_lshl_or_b32 %3, %4, %8, %3\n"
                "v_lshl_or_b32 %4, %5, %8, %4\n v_lshl_or_b32 %5, %6, %8, %5\n"
                "v_lshl_or_b32 %6, %7, %8, %6\n v_lshl_or_b32 %7, %0, %8, %7\n"
                : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                : "s"(s));
        } else if constexpr (KIND == 1) {  // v_and_b32
            asm volatile(
                "v_and_b32 %0, %1, %0\n v_and_b32 %1, %2, %1\n v_and_b32 %2, %3, %2\n v_and_b32 %3, %4, %3\n"
                "v_and_b32 %4, %5, %4\n v_and_b32 %5, %6, %5\n v_and_b32 %6, %7, %6\n v_and_b32 %7, %0, %7\n"
                : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
        } else if constexpr (KIND == 2) {  // v_fma_f32
            asm volatile(
                "v_fma_f32 %0, %1, %2, %0\n v_fma_f32 %1, %2, %3, %1\n v_fma_f32 %2, %3, %4, %2\n"
                "v_fma_f32 %3, %4, %5, %3\n v_fma_f32 %4, %5, %6, %4\n v_fma_f32 %5, %6, %7, %5\n"
                "v_fma_f32 %6, %7, %0, %6\n v_fma_f32 %7, %0, %1, %7\n"
                : "+v"(f0), "+v"(f1), "+v"(f2), "+v"(f3), "+v"(f4), "+v"(f5), "+v"(f6), "+v"(f7));
        } else if constexpr (KIND == 3) {  // v_bitop3_b32 (gfx950)
            asm volatile(
                "v_bitop3_b32 %0, %1, %2, %0 bitop3:0xf8\n v_bitop3_b32 %1, %2, %3, %1 bitop3:0xf8\n"
                "v_bitop3_b32 %2, %3, %4, %2 bitop3:0xf8\n v_bitop3_b32 %3, %4, %5, %3 bitop3:0xf8\n"
                "v_bitop3_b32 %4, %5, %6, %4 bitop3:0xf8\n v_bitop3_b32 %5, %6, %7, %5 bitop3:0xf8\n"
                "v_bitop3_b32 %6, %7, %0, %6 bitop3:0xf8\n v_bitop3_b32 %7, %0, %1, %7 bitop3:0xf8\n"
                : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
        } else {  // v_pk_add_u16 (2 x 16-bit per lane)
            asm volatile(
                "v_pk_add_u16 %0, %1, %0\n v_pk_add_u16 %1, %2, %1\n v_pk_add_u16 %2, %3, %2\n"
                "v_pk_add_u16 %3, %4, %3\n v_pk_add_u16 %4, %5, %4\n v_pk_add_u16 %5, %6, %5\n"
                "v_pk_add_u16 %6, %7, %6\n v_pk_add_u16 %7, %0, %7\n"
                : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
        }
    }
    uint32_t r = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ __float_as_uint(f0 + f1 + f2 + f3 + f4 + f5 + f6 + f7);
    if (r == 0x12345678u) out[blockIdx.x] = r;
}

template <int KIND>
static void run(const char* name, uint32_t* d, int num_cu) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    for (int wps = 1; wps <= 8; wps *= 2) {
        const int threads = 64 * 4 * wps;  // 4 SIMDs per CU, one block per CU
        hipLaunchKernelGGL(probe<KIND>, dim3(num_cu), dim3(threads), 0, 0, d, 1u);
        hipEventRecord(e0);
        for (int k = 0; k < 5; ++k) hipLaunchKernelGGL(probe<KIND>, dim3(num_cu), dim3(threads), 0, 0, d, 1u);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        const double instr_per_simd = (double)wps * N_ITERS * 8.0;
        const double ns_per_instr = ms / 5 * 1e6 / instr_per_simd;
        const double tops = (double)num_cu * 4 * wps * 64 * N_ITERS * 8.0 / (ms / 5 * 1e-3) / 1e12;
        printf("%-14s waves/SIMD=%d  %.3f ns per wave-instr per SIMD  (%.2f cyc @2.4GHz)  %.1f Tlane-op/s\n", name,
               wps, ns_per_instr, ns_per_instr * 2.4, tops);
    }
}

int main() {
    hipDeviceProp_t p; hipGetDeviceProperties(&p, 0);
    uint32_t* d; hipMalloc(&d, 4096 * 4);
    printf("CUs=%d clock=%d kHz\n", p.multiProcessorCount, p.clockRate);
    run<0>("v_lshl_or_b32", d, p.multiProcessorCount);
    run<1>("v_and_b32", d, p.multiProcessorCount);
    run<2>("v_fma_f32", d, p.multiProcessorCount);
    run<3>("v_bitop3_b32", d, p.multiProcessorCount);
    run<4>("v_pk_add_u16", d, p.multiProcessorCount);
    return 0;
}
